"""Does an initialised RCCL communicator slow the host-CPU work of a rank?

Run under torchrun with one rank on the GPU.  Times a fixed pure-Python loop
before the process group exists, after ``init_process_group("nccl")``, after
the first (communicator-creating) barrier, and after a gloo-only barrier on a
CPU subgroup; reports per-thread CPU seconds over an idle second after each
stage (a busy-polling runtime thread shows up there).  One JSON line.
"""
import json
import os
import time


def spin(n=2_000_000):
    t0 = time.perf_counter()
    x = 0
    for i in range(n):
        x += i & 7
    return round((time.perf_counter() - t0) * 1e3, 2)


def thread_cpu():
    out = {}
    for tid in os.listdir("/proc/self/task"):
        try:
            with open("/proc/self/task/%s/stat" % tid) as f:
                parts = f.read().rsplit(")", 1)[1].split()
            out[tid] = (int(parts[11]) + int(parts[12])) / os.sysconf("SC_CLK_TCK")
        except OSError:
            pass
    return out


def idle_cpu(sec=1.0):
    a = thread_cpu()
    time.sleep(sec)
    b = thread_cpu()
    busy = {t: round(b[t] - a.get(t, 0.0), 3) for t in b if b[t] - a.get(t, 0.0) > 0.02}
    return {"threads": len(b), "busy_threads_cpu_s": busy}


def main():
    res = {"spin_ms_before": spin(), "idle_before": idle_cpu()}
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
    dist.init_process_group("nccl")
    res["spin_ms_after_init"] = spin()
    gloo = dist.new_group(backend="gloo")
    dist.barrier(group=gloo)
    res["spin_ms_after_gloo_barrier"] = spin()
    res["idle_after_gloo_barrier"] = idle_cpu()
    dist.barrier(device_ids=[torch.cuda.current_device()])
    torch.cuda.synchronize()
    res["spin_ms_after_nccl_barrier"] = spin()
    res["idle_after_nccl_barrier"] = idle_cpu()
    time.sleep(2)
    res["spin_ms_2s_later"] = spin()
    if dist.get_rank() == 0:
        print(json.dumps(res), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
