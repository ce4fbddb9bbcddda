"""cProfile of warm bench steps (translate of samples/), sorted by argv[1] (default tottime)."""
import os, sys, time, tempfile, shutil, cProfile, pstats
sys.path.insert(0, os.environ.get('GRAFT_REPO_ROOT', '/root/repo'))
os.environ["M2K_NO_NETWORK"]="1"; os.environ["M2K_DISABLE_CNB"]="1"
from move2kube_amd import api
from move2kube_amd.utils import log
log.set_quiet()
work=tempfile.mkdtemp(); src=os.path.join(work,"samples"); shutil.copytree(os.path.join(os.environ.get('GRAFT_REPO_ROOT', '/root/repo'), 'samples'),src,symlinks=True)
with api.Session(qaskip=True) as s:
    for _ in range(5): s.translate(src, os.path.join(work,"out"), name="samples")
    pr=cProfile.Profile(); pr.enable()
    for _ in range(20): s.translate(src, os.path.join(work,"out"), name="samples")
    pr.disable()
    st=pstats.Stats(pr); st.sort_stats(sys.argv[1] if len(sys.argv)>1 else 'tottime').print_stats(40)
shutil.rmtree(work)
