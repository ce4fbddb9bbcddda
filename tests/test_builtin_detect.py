"""The in-process built-in detectors must agree with running the real scripts."""

import os
import shutil

import pytest

from move2kube_amd.parallel import builtin_detect, detect_pool

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _make_tree(base):
    trees = {
        "node": {"package.json": "{}"},
        "py": {"requirements.txt": "x", "app.py": "if __name__ == '__main__':\n  pass\n"},
        "py_nomain": {"setup.py": "x"},
        "gomod": {"go.mod": "module x"},
        "gosrc": {"sub/main.go": "package main"},
        "war": {"b.war": "x", "a.war": "y"},
        "mvn": {"pom.xml": "<p/>"},
        "gradle": {"build.gradle": "", "src/A.java": ""},
        "javasrc": {"x/y/A.java": ""},
        "php": {"deep/er/index.php": ""},
        "ruby": {"Gemfile": ""},
        "pipenv": {"Pipfile": ""},
        "ant": {"build.xml": ""},
        "empty": {},
        "dotgo": {".hidden.go": ""},
    }
    for name, files in trees.items():
        d = os.path.join(base, name)
        os.makedirs(d, exist_ok=True)
        for rel, content in files.items():
            p = os.path.join(d, rel)
            os.makedirs(os.path.dirname(p), exist_ok=True)
            with open(p, "w") as f:
                f.write(content)
    return [os.path.join(base, n) for n in sorted(trees)]


def test_builtin_matches_scripts(tmp_path, assets_dir, monkeypatch):
    targets = _make_tree(str(tmp_path / "src"))
    jobs = []
    for rel, script in sorted(builtin_detect.DETECTORS):
        for t in targets:
            jobs.append((os.path.join(assets_dir, rel), script, t))
    for job in jobs[:3]:
        assert builtin_detect.lookup(job[0], job[1]) is not None
    native_res = detect_pool.run_detect_jobs(jobs)
    monkeypatch.setenv("M2K_NATIVE_DETECT", "0")
    assert builtin_detect.lookup(jobs[0][0], jobs[0][1]) is None
    script_res = detect_pool.run_detect_jobs(jobs)
    mism = [(j, a.code, a.stdout, b.code, b.stdout) for j, a, b in zip(jobs, native_res, script_res)
            if (a.code == 0) != (b.code == 0) or (a.code == 0 and a.stdout != b.stdout)]
    assert mism == []


def test_builtin_matches_scripts_index_backed(tmp_path, assets_dir, monkeypatch):
    """Inside an fsindex scope the detectors answer ``test -f`` and the
    ``*.war`` glob from the directory index; edge cases must still agree with
    the scripts: markers that are directories, symlinks (to files, to
    directories, dangling), FIFOs, a symlinked source root, ``.war`` dirs."""
    from move2kube_amd.utils import fsindex
    base = str(tmp_path / "src")
    targets = _make_tree(base)
    extra = os.path.join(base, "edge")
    os.makedirs(os.path.join(extra, "package.json"))           # marker is a directory
    os.makedirs(os.path.join(extra, "z.war"))                  # .war directory
    with open(os.path.join(base, "real_gemfile"), "w") as f:
        f.write("")
    os.symlink(os.path.join(base, "real_gemfile"), os.path.join(extra, "Gemfile"))  # symlink to a file
    os.symlink(os.path.join(extra, "nowhere"), os.path.join(extra, "pom.xml"))     # dangling symlink
    os.symlink(os.path.join(base, "empty"), os.path.join(extra, "build.xml"))      # symlink to a dir
    os.mkfifo(os.path.join(extra, "Pipfile"))                                       # not a regular file
    os.symlink(os.path.join(base, "node"), os.path.join(base, "linkroot"))         # symlinked root
    targets += [extra, os.path.join(base, "linkroot")]
    jobs = [(os.path.join(assets_dir, rel), script, t)
            for rel, script in sorted(builtin_detect.DETECTORS) for t in targets]
    with fsindex.scope():
        fsindex.get_index(base)
        assert fsindex.peek_index(extra) is not None
        native_res = detect_pool.run_detect_jobs(jobs)
    monkeypatch.setenv("M2K_NATIVE_DETECT", "0")
    script_res = detect_pool.run_detect_jobs(jobs)
    mism = [(j, a.code, a.stdout, b.code, b.stdout) for j, a, b in zip(jobs, native_res, script_res)
            if (a.code == 0) != (b.code == 0) or (a.code == 0 and a.stdout != b.stdout)]
    assert mism == []


def test_modified_detector_is_not_shortcut(tmp_path, assets_dir):
    d = os.path.join(assets_dir, "dockerfiles", "nodejs")
    script = os.path.join(d, "m2kdfdetect.sh")
    with open(script, "a") as f:
        f.write("# local edit\n")
    assert builtin_detect.lookup(d, "m2kdfdetect.sh") is None


def test_user_detector_outside_assets_not_shortcut(tmp_path, assets_dir):
    d = tmp_path / "custom"
    shutil.copytree(os.path.join(assets_dir, "dockerfiles", "nodejs"), str(d))
    assert builtin_detect.lookup(str(d), "m2kdfdetect.sh") is None


@pytest.mark.reference
def test_detectors_match_reference_scripts(tmp_path, assets_dir):
    """Oracle: the reference's own detector scripts
    (``internal/assets/{dockerfiles,s2i}/*/m2k*detect.sh``), run as shell
    scripts, against our detectors (in-process built-ins) on every directory of
    the reference ``samples/`` corpus plus the synthetic edge trees above.
    Exit status (match / no match) and the JSON printed on a match must agree.

    The reference runs them with ``/bin/sh`` (``dockerfilecontainerizer.go:77``).
    Its python detectors use bash arrays, so they only work where ``/bin/sh``
    is bash (the reference's UBI8 image, macOS); the oracle runs them with
    ``bash`` to pin that behaviour (DEVIATIONS.md, "platform shell")."""
    import subprocess
    from conftest import ref_path
    if shutil.which("bash") is None:
        pytest.skip("bash not available")
    targets = _make_tree(str(tmp_path / "src"))
    samples = ref_path("samples")
    for dp, dns, _fns in os.walk(samples):
        dns.sort()
        targets.append(dp)
    jobs, ref = [], []
    for rel, script in sorted(builtin_detect.DETECTORS):
        ref_dir = ref_path("internal", "assets", rel)
        assert os.path.isfile(os.path.join(ref_dir, script)), rel
        for t in targets:
            jobs.append((os.path.join(assets_dir, rel), script, t))
            p = subprocess.run(["bash", script, t], cwd=ref_dir, stdout=subprocess.PIPE, stderr=subprocess.DEVNULL)
            ref.append((p.returncode, p.stdout.decode()))
    ours = detect_pool.run_detect_jobs(jobs)
    mism = [(j, rc, out, a.code, a.stdout) for j, (rc, out), a in zip(jobs, ref, ours)
            if (rc == 0) != (a.code == 0) or (rc == 0 and out != a.stdout)]
    assert mism == []
    assert sum(1 for rc, _ in ref if rc == 0) > 20  # the corpus really exercises the detectors


def test_packaged_assets_used_in_place_and_never_removed(tmp_path):
    """Without M2K_UNPACK_ASSETS the packaged detector tree is used read-only
    (no per-run copy); cleanup never deletes it and plans keep m2kassets/ paths."""
    from move2kube_amd import assets
    from move2kube_amd.utils.constants import ASSETS_DIR, settings
    saved = (settings.temp_path, settings.assets_path)
    try:
        tmp = assets.setup()
        assert settings.assets_path == assets.ASSETS_SRC
        assert os.path.relpath(settings.assets_path, settings.temp_path) == ASSETS_DIR
        scratch = assets.scratch_dir()
        assert os.path.isdir(scratch) and not scratch.startswith(assets.HERE)
        assets.cleanup(tmp)
        assert os.path.isfile(os.path.join(assets.ASSETS_SRC, "dockerfiles", "nodejs", "m2kdfdetect.sh"))
        assert not os.path.exists(scratch)
    finally:
        settings.temp_path, settings.assets_path = saved


def test_builtin_matches_scripts_on_random_trees(tmp_path, assets_dir, monkeypatch):
    """Random trees of detector marker files (nested, hidden, dangling
    symlinks, directories named like markers, contents that are not UTF-8):
    every built-in detector answers as its shell script does."""
    import random
    names = ["package.json", "pom.xml", "build.gradle", "requirements.txt", "setup.py", "Pipfile", "Gemfile", "go.mod",
             "main.go", ".h.go", "a.war", "a b.war", "A.java", "index.php", "build.xml", "composer.json", "manage.py",
             "main.py", "app.py", "Gemfile.lock", "config.ru", "x.GO", "X.WAR", "package.JSON", "sub", "src"]
    contents = ["", "{}", '{"scripts": {"start": "node x"}}', "if __name__ == '__main__':\n  run()\n",
                "module example.com/x\n", "package main\n", "flask\n", "\xff\xfe"]
    rnd = random.Random(11)
    for it in range(40):
        targets = []
        for t in range(6):
            d = tmp_path / ("i%d" % it) / ("t%d" % t)
            d.mkdir(parents=True)
            for _ in range(rnd.randint(0, 5)):
                p = d / rnd.choice(["", "sub/", "src/main/", ".hidden/"]) / rnd.choice(names)
                try:
                    p.parent.mkdir(parents=True, exist_ok=True)
                except (FileExistsError, NotADirectoryError):
                    continue
                if os.path.lexists(p):
                    continue
                if rnd.random() < 0.1:
                    p.mkdir()
                else:
                    p.write_text(rnd.choice(contents), encoding="latin-1")
            if rnd.random() < 0.1:
                os.symlink("/nonexistent", str(d / rnd.choice(names)))
            targets.append(str(d))
        jobs = [(os.path.join(assets_dir, rel), script, t) for rel, script in sorted(builtin_detect.DETECTORS)
                for t in targets]
        monkeypatch.delenv("M2K_NATIVE_DETECT", raising=False)
        ours = detect_pool.run_detect_jobs(jobs)
        monkeypatch.setenv("M2K_NATIVE_DETECT", "0")
        scripts = detect_pool.run_detect_jobs(jobs)
        assert [(j, a.code == 0, a.stdout if a.code == 0 else None) for j, a in zip(jobs, ours)] == \
            [(j, b.code == 0, b.stdout if b.code == 0 else None) for j, b in zip(jobs, scripts)]
