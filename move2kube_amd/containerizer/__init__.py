"""Containerization: Dockerfile / S2I / CNB / Reuse (registry) plus Manual and
ReuseDockerfile (called directly), and the CNB runtime providers."""

from .base import ContainerizationOption, Containerizers, ContainerizerError  # noqa: F401
