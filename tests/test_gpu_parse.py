"""libffm text parsed on the device (csrc/hip/kernels_parse.hip via
Engine.parse_text / data.textstream.TextStream) vs the native host parser
(csrc/io/reader.cpp, itself checked against the reference's rules in
test_reader.py): bit-equal keys (std::hash of the feature text), field ids,
labels and row offsets, with the reference's block carry-over protocol --
on the bundled CRLF data, on a generated Criteo-shaped file with multi-valued
fields, and on malformed / edge-case lines."""
import os

import numpy as np
import pytest
import torch

from conftest import DATA
from xflow_amd import native
from xflow_amd.config import EngineConfig, ModelConfig, OptimConfig
from xflow_amd.engine import Engine
from xflow_amd.data.textstream import TextBlocks, parse_text_file

EDGE = (b"1\t0:a:1 1:bb:1 2:ccc\r\n"          # 2-part token at a CRLF end
        b"no tab here\n"                        # no row
        b"0.5\t3:x:1  4:y:1 :z:1 5:\r\n"        # double space, empty field, empty fid
        b"0\t\n"                                # a row without features
        b"-1e-8\t7:0123456789abcdefghij:0.5 8:k\n"  # long fid (> 8 bytes), 2-part at LF
        b"\t9:q:1 nocolon 10:r:1\n"             # empty label, token without ':'
        b"  1.0e0\t+11:s:1 -2:t:1 1.9:u:1\n"    # atof of labels / field ids
        b"inf\t12:v\n"
        b"1\t13:w:1")                           # no final newline


def _host_blocks(path, block_bytes):
    r = native.load().BlockReader(path, block_bytes)
    out = []
    while True:
        b = r.next()
        if b is None:
            break
        out.append({k: np.asarray(b[k]) for k in ("keys", "labels", "row_ptr", "fgid")})
    return out


def _engine(device):
    return Engine(ModelConfig(kind="lr"), OptimConfig(), EngineConfig(table_log2_cap=12),
                  device=device)


def _compare(path, device, block_bytes):
    want = _host_blocks(path, block_bytes)
    got = parse_text_file(_engine(device), path, block_bytes)
    assert len(got) == len(want)
    for g, w in zip(got, want):
        assert g["rows"] == len(w["labels"])
        np.testing.assert_array_equal(g["keys"].view(np.uint64), w["keys"].view(np.uint64))
        np.testing.assert_array_equal(g["fgid"], w["fgid"])
        np.testing.assert_array_equal(g["labels"], w["labels"])
        np.testing.assert_array_equal(g["row_ptr"], w["row_ptr"])
        lens = np.diff(w["row_ptr"])
        assert g["nnz_per_row"] == (int(lens[0]) if len(lens) and (lens == lens[0]).all() else 0)
    return got


def _gen(path, rows, multi=True, seed=3):
    rng = np.random.default_rng(seed)
    with open(path, "w") as f:
        for i in range(rows):
            toks = []
            for j in range(39):
                for _ in range(rng.integers(1, 3) if multi and j >= 36 else 1):
                    toks.append("%d:%d:1" % (j, int(min(rng.zipf(1.2), 10 ** 7)) * 64 + j))
            f.write("%d\t%s\n" % (int(rng.random() < 0.25), " ".join(toks)))


@pytest.fixture(scope="module")
def gen_file(tmp_path_factory):
    p = str(tmp_path_factory.mktemp("ffm") / "criteo-00000")
    _gen(p, 3000)
    return p


@pytest.mark.parametrize("threads", [1, 4])
def test_text_blocks_protocol_matches_block_reader(gen_file, threads, monkeypatch):
    """Block boundaries (and the carried tails) equal BlockReader's, with
    one reader or parallel positional reads of small pieces."""
    monkeypatch.setattr(TextBlocks, "min_piece", 1000)
    for bb in (4096, 65536, 1 << 20):
        want = [len(b["labels"]) for b in _host_blocks(gen_file, bb)]
        tb = TextBlocks(gen_file, bb, read_threads=threads)
        buf = np.empty(bb + 16, np.uint8)
        got = []
        while True:
            n = tb.read_into(buf)
            if n == 0:
                break
            got.append(bytes(buf[:n]).count(b"\n"))
        assert got == want


@pytest.mark.parametrize("block_bytes", [2 << 20, 4096])
def test_cpu_parse_text_equals_host_reader(tmp_path, gen_file, block_bytes):
    _compare(os.path.join(DATA, "small_train-00000"), torch.device("cpu"), block_bytes)
    _compare(gen_file, torch.device("cpu"), block_bytes)


@pytest.mark.gpu
@pytest.mark.parametrize("block_bytes", [2 << 20, 4096, 1 << 16])
def test_gpu_parse_bundled_and_generated(gpu_device, gen_file, block_bytes):
    _compare(os.path.join(DATA, "small_train-00000"), gpu_device, block_bytes)
    _compare(os.path.join(DATA, "small_test-00000"), gpu_device, block_bytes)
    _compare(gen_file, gpu_device, block_bytes)


@pytest.mark.gpu
def test_gpu_parse_edge_lines(gpu_device, tmp_path):
    p = str(tmp_path / "edge-00000")
    with open(p, "wb") as f:
        f.write(EDGE)
    got = _compare(p, gpu_device, 1 << 20)
    assert got[0]["rows"] == 8


@pytest.mark.gpu
def test_trainer_gpu_parse_equals_host_parse(gpu_device, tmp_path):
    """The Trainer fed by the GPU tokeniser trains the same model as the one
    fed by the host parser (bundled data, 8 slices, reference blocks)."""
    from xflow_amd.config import TrainConfig
    from xflow_amd.trainer import Trainer

    preds = []
    for gp in (False, True):
        d = tmp_path / ("gpu" if gp else "host")
        cfg = TrainConfig(train_prefix=os.path.join(DATA, "small_train"),
                          test_prefix=os.path.join(DATA, "small_test"), epochs=3, threads=8,
                          gpu_parse=gp, pred_dir=str(d),
                          model=ModelConfig(kind="fm", v_dim=4),
                          engine=EngineConfig(table_log2_cap=14))
        Trainer(cfg, device=gpu_device).train()
        preds.append(np.loadtxt(d / "pred_0_0.txt"))
    np.testing.assert_array_equal(preds[0], preds[1])
