"""Common utilities: constants, logging, go-yaml-compatible YAML IO, a Go
text/template interpreter, the single-walk file index, git discovery, naming
and hashing helpers, tar helpers and SSH key/known-hosts handling."""
