# Cold-start diagnosis on the GPU box into gpurun_out/$RUN/: stale bytecode
# caches, interpreter floors with and without site, -X importtime of the floor
# and of a cold translate; then the smoke() kernels under rocprofv3 (CSV stats).
set -e
cd $GRAFT_REPO_ROOT
RUN=${RUN:-cold_diag}
OUT=gpurun_out/$RUN
mkdir -p $OUT
export M2K_NO_NETWORK=1 M2K_DISABLE_CNB=1
timeout -k 10 60 python -u scripts/pyc_diag.py > $OUT/pyc_diag.json 2> $OUT/pyc_diag.err
python -X importtime -c pass 2> $OUT/importtime_floor.txt
python -X importtime -S -c pass 2> $OUT/importtime_floor_nosite.txt
timeout -k 10 120 python - > $OUT/floors.json <<'EOF'
import json, os, shutil, statistics, subprocess, sys, tempfile, time
w = tempfile.mkdtemp()
shutil.copytree("samples/golang", os.path.join(w, "src"))
env = dict(os.environ, PYTHONPATH=os.getcwd())
def p50(argv, n=11):
    ws = []
    for _ in range(n):
        shutil.rmtree(os.path.join(w, "out"), ignore_errors=True)
        t0 = time.perf_counter()
        subprocess.run(argv, cwd=w, env=env, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, check=True)
        ws.append(time.perf_counter() - t0)
    return round(statistics.median(ws) * 1e3, 2)
tr = ["-m", "move2kube_amd", "translate", "-s", "src", "-o", "out", "--qaskip"]
print(json.dumps({"floor": p50([sys.executable, "-c", "pass"]), "floor_S": p50([sys.executable, "-S", "-c", "pass"]),
                  "floor_I": p50([sys.executable, "-I", "-c", "pass"]),
                  "translate": p50([sys.executable] + tr), "version": p50([sys.executable, "-m", "move2kube_amd", "version"])}))
EOF
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/rocprof -o smoke -- python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/rocprof_smoke.log 2>&1
echo done
