"""Data models: plan, QA problems/caches, collection kinds, helm values,
version info and the intermediate representation (IR)."""
