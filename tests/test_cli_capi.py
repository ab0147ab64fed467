"""Entry points: the native xflow_lr binary, the Python CLI, the compat
launch scripts and the C API (libxflow_api.so: XFCreate / XFStartTrain)."""
import ctypes
import os
import subprocess
import sys

import pytest

from conftest import DATA, ROOT

TRAIN = os.path.join(DATA, "small_train")
TEST = os.path.join(DATA, "small_test")
ENV = dict(os.environ, PYTHONPATH=ROOT, HIP_VISIBLE_DEVICES="", XFLOW_DEVICE="-1")


def _run(cmd, cwd, timeout=300, env=ENV):
    r = subprocess.run(cmd, cwd=cwd, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


def _lines(out):
    return [l for l in out.splitlines() if l.strip()]


def test_native_binary_matches_reference_output(tmp_path):
    out = _run([os.path.join(ROOT, "build", "bin", "xflow_lr"), TRAIN, TEST, "0", "30",
                "--threads", "8"], tmp_path)
    ls = _lines(out)
    assert ls[0].strip() == "start LR"
    assert ls[1] == "my rank is = 0"
    assert "epoch : 29" in ls
    i = ls.index("LR AUC: ")
    assert ls[i + 1].startswith("logloss: -0.") and "\tauc = 0.5" in ls[i + 1]
    assert ls[-1] == "train end......"
    assert len(open(tmp_path / "pred_0_0.txt").read().splitlines()) == 200


def test_native_binary_usage_and_roles(tmp_path):
    r = subprocess.run([os.path.join(ROOT, "build", "bin", "xflow_lr")], capture_output=True,
                       text=True, env=ENV)
    assert r.returncode == 1 and "run_ps_local.sh" in r.stdout
    env = dict(ENV, DMLC_ROLE="server")
    out = _run([os.path.join(ROOT, "build", "bin", "xflow_lr"), TRAIN, TEST, "0", "1"],
               tmp_path, env=env)
    assert "init server success" in out


def test_python_cli_equals_native(tmp_path):
    a = _run([os.path.join(ROOT, "build", "bin", "xflow_lr"), TRAIN, TEST, "1", "5",
              "--threads", "8"], tmp_path / ".." if False else tmp_path)
    os.rename(tmp_path / "pred_0_0.txt", tmp_path / "native.txt")
    b = _run([sys.executable, "-m", "xflow_amd.cli", TRAIN, TEST, "1", "5", "--threads", "8",
              "--cpu"], tmp_path)
    la = [l for l in _lines(a) if l.startswith("logloss")]
    lb = [l for l in _lines(b) if l.startswith("logloss")]
    assert la == lb
    assert open(tmp_path / "native.txt").read() == open(tmp_path / "pred_0_0.txt").read()


def test_run_ps_local_script_three_workers(tmp_path):
    env = dict(ENV, XFLOW_FLAGS="--threads 8")
    out = _run(["bash", os.path.join(ROOT, "run_ps_local.sh"), "0", "5", "3"], tmp_path,
               env=env)
    assert out.count("train end......") == 3
    assert out.count("init server success") == 1
    assert sum(1 for l in _lines(out) if l.startswith("logloss: ")) == 1


def test_cli_checkpoint_save_and_resume(tmp_path):
    ck = str(tmp_path / "ck")
    _run([sys.executable, "-m", "xflow_amd.cli", TRAIN, TEST, "0", "3", "--threads", "8",
          "--cpu", "--save", ck, "--metrics", str(tmp_path / "m.jsonl")], tmp_path)
    assert os.path.exists(os.path.join(ck, "meta.json"))
    assert os.path.exists(os.path.join(ck, "shard-00000-of-00001.xftb"))
    out = _run([sys.executable, "-m", "xflow_amd.cli", TRAIN, TEST, "0", "0", "--threads", "8",
                "--cpu", "--load", ck], tmp_path)
    first = [l for l in open(tmp_path / "pred_0_0.txt")]
    assert len(first) == 200 and "logloss: " in out
    recs = [l for l in open(tmp_path / "m.jsonl")]
    assert any('"event": "epoch"' in r for r in recs) and any('"event": "eval"' in r for r in recs)


def test_c_api(tmp_path):
    lib = ctypes.CDLL(os.path.join(ROOT, "build", "lib", "libxflow_api.so"))
    lib.XFCreateEx.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_char_p, ctypes.c_char_p,
                               ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]
    lib.XFGetLastError.restype = ctypes.c_char_p
    h = ctypes.c_void_p()
    cwd = os.getcwd()
    os.chdir(tmp_path)
    try:
        assert lib.XFCreateEx(ctypes.byref(h), TRAIN.encode(), TEST.encode(), 0, 10, 8, -1) == 0
        assert lib.XFStartTrain(ctypes.byref(h)) == 0, lib.XFGetLastError()
        ll, auc = ctypes.c_double(), ctypes.c_double()
        assert lib.XFPredict(ctypes.byref(h), ctypes.byref(ll), ctypes.byref(auc)) == 0
        assert -1.0 < ll.value < -0.5 and 0.5 < auc.value < 0.7
        assert lib.XFSave(ctypes.byref(h), str(tmp_path / "t.xftb").encode()) == 0
        assert lib.XFFree(ctypes.byref(h)) == 0 and not h.value
        bad = ctypes.c_void_p()
        assert lib.XFCreate(ctypes.byref(bad), b"/nonexistent/x", TEST.encode()) == 0
        assert lib.XFStartTrain(ctypes.byref(bad)) == -1
        assert b"error" in lib.XFGetLastError()
        lib.XFFree(ctypes.byref(bad))
    finally:
        os.chdir(cwd)


def test_local_sh_records_pids_and_stop_sh_kills_them(tmp_path):
    """scripts/local.sh writes every process it starts to the pid file and
    scripts/stop.sh stops exactly those (the reference's stop.sh kill -9s
    every xflow_lr by name)."""
    import subprocess
    import time

    pidfile = tmp_path / "pids"
    env = dict(os.environ, XFLOW_PIDFILE=str(pidfile))
    launcher = subprocess.Popen(["bash", os.path.join(ROOT, "scripts", "local.sh"), "1", "2",
                                 "sleep", "60"], env=env, stdout=subprocess.PIPE,
                                stderr=subprocess.STDOUT)
    try:
        for _ in range(100):
            if pidfile.exists() and len(pidfile.read_text().split()) == 4:
                break
            time.sleep(0.05)
        pids = [int(p) for p in pidfile.read_text().split()]
        assert len(pids) == 4  # scheduler + 1 server + 2 workers
        for p in pids:
            os.kill(p, 0)  # alive
        out = subprocess.run(["bash", os.path.join(ROOT, "scripts", "stop.sh")], env=env,
                             capture_output=True, text=True, timeout=30)
        assert "stopped 4" in out.stdout, out.stdout + out.stderr
        assert launcher.wait(timeout=30) != 0  # its workers were killed
        for p in pids:
            with pytest.raises(ProcessLookupError):
                os.kill(p, 0)
        assert not pidfile.exists()
    finally:
        if launcher.poll() is None:
            launcher.kill()


GPU_ENV = dict(os.environ, PYTHONPATH=ROOT, XFLOW_DEVICE="0")


def _eval_line(out):
    line = [l for l in _lines(out) if l.startswith("logloss: ")][-1]
    ll = float(line.split("\t")[0].split()[1])
    auc = float(line.split("auc = ")[1].split("\t")[0])
    return ll, auc


@pytest.mark.gpu
@pytest.mark.parametrize("model", ["0", "1", "2"])
def test_native_binary_gpu_matches_cpu(tmp_path, model):
    """build/bin/xflow_lr on the HIP backend (double-buffered H2D staging on a
    copy queue) trains the same model as on the native CPU backend."""
    binp = os.path.join(ROOT, "build", "bin", "xflow_lr")
    (tmp_path / "cpu").mkdir()
    (tmp_path / "gpu").mkdir()
    a = _run([binp, TRAIN, TEST, model, "5", "--threads", "8"], tmp_path / "cpu")
    b = _run([binp, TRAIN, TEST, model, "5", "--threads", "8", "--device", "0"],
             tmp_path / "gpu", env=GPU_ENV)
    (lla, auca), (llb, aucb) = _eval_line(a), _eval_line(b)
    assert abs(lla - llb) <= 1e-4 * abs(lla) and abs(auca - aucb) <= 2e-3
    pa = [[float(x) for x in l.split()] for l in open(tmp_path / "cpu" / "pred_0_0.txt")]
    pb = [[float(x) for x in l.split()] for l in open(tmp_path / "gpu" / "pred_0_0.txt")]
    import numpy as np

    np.testing.assert_allclose(np.array(pb), np.array(pa), rtol=1e-4, atol=1e-5)


@pytest.mark.gpu
def test_c_api_gpu_matches_cpu(tmp_path):
    lib = ctypes.CDLL(os.path.join(ROOT, "build", "lib", "libxflow_api.so"))
    lib.XFCreateEx.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_char_p, ctypes.c_char_p,
                               ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]
    lib.XFGetLastError.restype = ctypes.c_char_p
    res = []
    cwd = os.getcwd()
    for dev in (-1, 0):
        d = tmp_path / str(dev)
        d.mkdir()
        os.chdir(d)
        try:
            h = ctypes.c_void_p()
            assert lib.XFCreateEx(ctypes.byref(h), TRAIN.encode(), TEST.encode(), 0, 10, 8,
                                  dev) == 0
            assert lib.XFStartTrain(ctypes.byref(h)) == 0, lib.XFGetLastError()
            ll, auc = ctypes.c_double(), ctypes.c_double()
            assert lib.XFPredict(ctypes.byref(h), ctypes.byref(ll), ctypes.byref(auc)) == 0
            res.append((ll.value, auc.value))
            assert lib.XFFree(ctypes.byref(h)) == 0
        finally:
            os.chdir(cwd)
    (la, aa), (lb, ab) = res
    assert abs(la - lb) <= 1e-4 * abs(la) and abs(aa - ab) <= 2e-3


def test_cli_async_staleness_and_fixed_table_flags(tmp_path):
    """--async --staleness 2 on 2 gloo ranks trains and predicts; with a
    fixed tiny table (--no-table-grow) the run fails fast with an overflow."""
    env = dict(os.environ, PYTHONPATH=ROOT, HIP_VISIBLE_DEVICES="")
    base = ["bash", os.path.join(ROOT, "run_ps_local.sh"), "0", "2", "2"]
    r = subprocess.run(base, cwd=tmp_path, capture_output=True, text=True, timeout=240,
                       env=dict(env, XFLOW_FLAGS="--threads 4 --cpu --async --staleness 2"))
    assert r.returncode == 0, r.stderr[-2000:]
    assert "logloss:" in r.stdout
    r = subprocess.run([sys.executable, "-m", "xflow_amd.cli", os.path.join(DATA, "small_train"),
                        os.path.join(DATA, "small_test"), "0", "1", "--threads", "4", "--cpu",
                        "--log2-cap", "6", "--no-table-grow"], cwd=tmp_path, capture_output=True,
                       text=True, timeout=240, env=env)
    assert r.returncode != 0 and "overflow" in r.stderr, r.stderr[-2000:]
    r = subprocess.run([sys.executable, "-m", "xflow_amd.cli", os.path.join(DATA, "small_train"),
                        os.path.join(DATA, "small_test"), "0", "1", "--threads", "4", "--cpu",
                        "--log2-cap", "6"], cwd=tmp_path, capture_output=True, text=True,
                       timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
