"""docker-compose parsing: v1/v2 (libcompose semantics) and v3 (docker/cli semantics)."""
