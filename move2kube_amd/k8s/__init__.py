"""Kubernetes object layer: type registry/decoding, Go encoding/json
marshalling rules, and GroupVersion conversion."""
