"""Parallel execution: the detect-script process pool and the multi-rank
(torch.distributed) harness used by the benchmark."""
