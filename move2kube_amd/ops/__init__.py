"""Native and GPU operators (see ``csrc/``): file-tree walk, Dockerfile sniffing,
process pool, naming hashes and batched fuzzy matching (CPU + MI355X)."""
