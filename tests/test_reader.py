"""libffm block reader: parse rules of load_data_from_disk.cc:103-210 on the
bundled data (CRLF, multi-valued fields 16/17), std::hash keys, block carry-over,
and the reference-compatible LoadData API."""
import os

import numpy as np
import pytest

from conftest import DATA
from xflow_amd.testing.hashing import std_hash


def py_parse(path):
    """Independent Python parse of a libffm file (reference rules)."""
    rows = []
    with open(path, "rb") as f:
        for line in f.read().split(b"\n"):
            if b"\t" not in line:
                continue
            lab, rest = line.split(b"\t", 1)
            y = 1 if float(lab) > 1e-7 else 0
            feats = []
            for tok in rest.split(b" "):
                if not tok or b":" not in tok:
                    continue
                parts = tok.split(b":")
                feats.append((int(float(parts[0])), std_hash(parts[1])))
            rows.append((y, feats))
    return rows


def read_all(native, path, block):
    r = native.BlockReader(path, block)
    out = []
    while True:
        b = r.next()
        if b is None:
            break
        rp = b["row_ptr"]
        for i in range(len(b["labels"])):
            s, e = rp[i], rp[i + 1]
            out.append((int(b["labels"][i]), list(zip(b["fgid"][s:e].tolist(),
                                                        b["keys"][s:e].tolist()))))
    return out


@pytest.mark.parametrize("name", ["small_train-00000", "small_test-00000"])
def test_bundled_files_parse_like_reference(native, name):
    path = os.path.join(DATA, name)
    want = py_parse(path)
    got = read_all(native, path, 2 << 20)
    assert len(got) == 200
    assert got == want


def test_label_counts_and_fields(native):
    tr = read_all(native, os.path.join(DATA, "small_train-00000"), 2 << 20)
    te = read_all(native, os.path.join(DATA, "small_test-00000"), 2 << 20)
    assert sum(y for y, _ in tr) == 48 and sum(y for y, _ in te) == 46
    fg = {g for _, f in tr for g, _ in f}
    assert fg == set(range(18))
    # fields 16/17 are multi-valued in some rows
    assert any(sum(1 for g, _ in f if g == 16) > 1 for _, f in tr + te)


@pytest.mark.parametrize("block", [600, 1000, 4096, 65536])  # >= longest line
def test_block_carry_over_preserves_rows(native, block):
    path = os.path.join(DATA, "small_train-00000")
    assert read_all(native, path, block) == read_all(native, path, 2 << 20)


def test_crlf_value_ignored_and_key_is_fid_text(native):
    b = native.parse_libffm(b"1\t0:abc:0.5 3:xyz:1\r\n0\t2:abc:7\n")
    assert b["labels"].tolist() == [1.0, 0.0]
    assert b["row_ptr"].tolist() == [0, 2, 3]
    assert b["keys"].tolist() == [std_hash("abc"), std_hash("xyz"), std_hash("abc")]
    assert b["fgid"].tolist() == [0, 3, 2]


def test_label_threshold_and_empty_rows(native):
    b = native.parse_libffm(b"0.0000001\t1:a:1\n0.5\t\n-1\t2:b:1\nnotab line\n")
    assert b["labels"].tolist() == [0.0, 1.0, 0.0]
    assert b["row_ptr"].tolist() == [0, 1, 1, 2]


def test_loaddata_compat_api(native):
    ld = native.LoadData(os.path.join(DATA, "small_test-00000"), 4 << 20)
    ld.load_minibatch_hash_data_fread()
    assert len(ld.fea_matrix) == 200 and len(ld.label) == 200
    ref = py_parse(os.path.join(DATA, "small_test-00000"))
    assert [(y, [tuple(t) for t in f]) for y, f in zip(ld.label, ld.fea_matrix)] == \
        [(y, f) for y, f in ref]
    ld.load_minibatch_hash_data_fread()
    assert len(ld.fea_matrix) == 0


def test_prefetch_reader_equals_block_reader(native):
    path = os.path.join(DATA, "small_train-00000")
    a, b = native.BlockReader(path, 1500), native.PrefetchReader(path, 1500)
    while True:
        x, y = a.next(), b.next()
        if x is None:
            assert y is None
            break
        for k in ("row_ptr", "keys", "fgid", "labels"):
            np.testing.assert_array_equal(x[k], y[k])


def test_missing_file_raises(native):
    with pytest.raises(RuntimeError):
        native.BlockReader("/nonexistent/file-00000", 1024)


def test_parallel_parse_equals_serial(tmp_path, native):
    """Blocks parsed on several threads (split at line boundaries) equal the
    serial parse bit for bit, including the block carry-over."""
    src = open(os.path.join(DATA, "small_train-00000"), "rb").read()
    path = tmp_path / "big-00000"
    path.write_bytes(src * 100)  # ~2.6 MB: several 1 MB blocks, >= 256 KB per thread
    out = {}
    for threads in (1, 4):
        r = native.BlockReader(str(path), 1 << 20)
        r.parse_threads = threads
        blocks = []
        while True:
            b = r.next()
            if b is None:
                break
            blocks.append(b)
        out[threads] = blocks
    assert len(out[1]) == len(out[4]) >= 3
    for a, b in zip(out[1], out[4]):
        for k in ("row_ptr", "keys", "fgid", "labels"):
            np.testing.assert_array_equal(a[k], b[k])
    assert sum(len(b["labels"]) for b in out[4]) == 200 * 100


def test_xfb_shard_blocks_equal_text_reader(tmp_path, native):
    """An .xfb shard (binfmt.convert) holds exactly what the text reader parses."""
    from xflow_amd.data import binfmt

    src = os.path.join(DATA, "small_train-00000")
    dst = str(tmp_path / "s.xfb")
    info = binfmt.convert(src, dst, block_bytes=1000, threads=2)
    r = native.BlockReader(src, 1 << 20)
    b = r.next()
    assert r.next() is None
    assert info == {"rows": len(b["labels"]), "nnz": len(b["keys"])}
    s = binfmt.ShardReader(dst, block_rows=37)
    parts = []
    while True:
        x = s.next()
        if x is None:
            break
        assert len(x["labels"]) <= 37 and x["row_ptr"][0] == 0
        assert x["row_ptr"][-1] == len(x["keys"])
        parts.append(x)
    np.testing.assert_array_equal(np.concatenate([p["labels"] for p in parts]), b["labels"])
    np.testing.assert_array_equal(np.concatenate([p["keys"] for p in parts]),
                                  np.asarray(b["keys"]).view(np.uint64))
    np.testing.assert_array_equal(np.concatenate([p["fgid"] for p in parts]), b["fgid"])
    lens = np.concatenate([np.diff(p["row_ptr"]) for p in parts])
    np.testing.assert_array_equal(lens, np.diff(b["row_ptr"]))
    assert binfmt.max_block(dst, 37)[0] == 37


def test_xfb_write_roundtrip_and_bad_magic(tmp_path):
    from xflow_amd.data import binfmt

    rp = np.array([0, 2, 2, 5])
    keys = np.arange(5, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)
    binfmt.write(str(tmp_path / "a.xfb"), np.array([1, 0, 1]), rp, keys)
    s = binfmt.Shard(str(tmp_path / "a.xfb"))
    assert (s.rows, s.nnz) == (3, 5)
    np.testing.assert_array_equal(s.keys, keys)
    np.testing.assert_array_equal(s.fgid, np.zeros(5, np.int32))
    with pytest.raises(ValueError):
        binfmt.write(str(tmp_path / "b.xfb"), np.array([1, 0]), rp, keys)
    (tmp_path / "c.xfb").write_bytes(b"NOTASHARD" * 8)
    with pytest.raises(ValueError):
        binfmt.Shard(str(tmp_path / "c.xfb"))


@pytest.mark.parametrize("kind", ["lr", "fm"])
def test_trainer_on_xfb_equals_text(tmp_path, kind):
    """Training from .xfb shards (text files absent) predicts exactly like
    training from the libffm text (one block per epoch in both)."""
    import shutil

    import torch

    from xflow_amd.config import EngineConfig, ModelConfig, TrainConfig
    from xflow_amd.data import binfmt
    from xflow_amd.trainer import Trainer

    preds = []
    for mode in ("text", "xfb"):
        d = tmp_path / mode
        d.mkdir()
        for name in ("small_train-00000", "small_test-00000"):
            if mode == "text":
                shutil.copy(os.path.join(DATA, name), d / name)
            else:
                binfmt.convert(os.path.join(DATA, name), str(d / (name + ".xfb")))
        cfg = TrainConfig(train_prefix=str(d / "small_train"), test_prefix=str(d / "small_test"),
                          epochs=3, threads=8, pred_dir=str(d), model=ModelConfig(kind=kind),
                          engine=EngineConfig(table_log2_cap=14))
        Trainer(cfg, device=torch.device("cpu")).train()
        preds.append(np.loadtxt(d / "pred_0_0.txt"))
    assert len(preds[1]) == 200
    np.testing.assert_array_equal(preds[0], preds[1])


def _fixed_width_shards(d, rows=300, F=12, seed=0, hash32=False, compact="auto", csr=False):
    """Uniform-width train/test .xfb shards (every row holds F features);
    hash32: keys below 2^32 (stored compact unless compact="off"); csr: rows
    of F-1 or F features."""
    from xflow_amd.data import binfmt

    rng = np.random.default_rng(seed)
    for name, n in (("tr-00000.xfb", rows), ("te-00000.xfb", rows // 3)):
        keys = (rng.zipf(1.3, size=n * F).astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15)
                + np.tile(np.arange(F, dtype=np.uint64), n))
        if hash32:
            keys = keys >> np.uint64(32)
        fg = np.tile(np.arange(F, dtype=np.int32), n)
        rp = np.arange(n + 1) * F
        if csr:  # drop the last feature of every third row
            keep = np.ones(n * F, bool)
            keep[np.arange(0, n, 3) * F + F - 1] = False
            keys, fg = keys[keep], fg[keep]
            rp = np.concatenate([[0], np.cumsum(np.where(np.arange(n) % 3 == 0, F - 1, F))])
        binfmt.write(str(d / name), (rng.random(n) < 0.3).astype(np.float32), rp, keys, fg,
                     compact=compact)


def _train_preds(d, tag, device="cpu", **kw):
    import torch

    from xflow_amd.config import EngineConfig, ModelConfig, TrainConfig
    from xflow_amd.trainer import Trainer

    out = d / tag
    out.mkdir()
    model = ModelConfig(kind=kw.pop("kind", "lr"))
    cfg = TrainConfig(train_prefix=str(d / "tr"), test_prefix=str(d / "te"), epochs=3, threads=4,
                      pred_dir=str(out), model=model, engine=EngineConfig(table_log2_cap=14),
                      block_rows=kw.pop("block_rows", 64), **kw)
    Trainer(cfg, device=torch.device(device)).train()
    return np.loadtxt(out / "pred_0_0.txt")


@pytest.mark.parametrize("kind", ["lr", "fm", "mvm"])
def test_fixed_width_blocks_train_like_csr(tmp_path, kind):
    """Uniform-width blocks go through the field-major path and predict like
    the same rows fed as CSR."""
    _fixed_width_shards(tmp_path)
    a = _train_preds(tmp_path, "fm", kind=kind)
    b = _train_preds(tmp_path, "csr", kind=kind, fixed_width=False)
    assert len(a) == 100
    np.testing.assert_allclose(a, b, rtol=1e-5, atol=1e-6)


def test_resident_epochs_equal_streamed(tmp_path):
    """--resident (first epoch's batches kept on the device) trains exactly
    like re-reading the shard every epoch."""
    _fixed_width_shards(tmp_path)
    a = _train_preds(tmp_path, "stream")
    b = _train_preds(tmp_path, "resident", resident=True)
    np.testing.assert_array_equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("fixed", [True, False])
def test_block_stream_trainer_gpu_matches_cpu(gpu_device, tmp_path, fixed):
    """GPU trainer fed through the pinned/copy-stream BlockStream (and the
    resident cache) predicts like the CPU trainer."""
    _fixed_width_shards(tmp_path, rows=3000)
    a = _train_preds(tmp_path, "cpu", fixed_width=fixed, block_rows=512)
    b = _train_preds(tmp_path, "gpu", device=str(gpu_device), fixed_width=fixed, block_rows=512)
    c = _train_preds(tmp_path, "gpu_res", device=str(gpu_device), fixed_width=fixed,
                     block_rows=512, resident=True)
    np.testing.assert_allclose(a, b, rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(b, c, rtol=1e-4, atol=1e-5)  # float atomics: not bitwise


def test_xfb_compact_keys_roundtrip(tmp_path):
    """Keys below 2^32 are stored as u32 (version 2, flag bit 1): same values,
    half the key bytes; compact=False keeps the u64 layout."""
    from xflow_amd.data import binfmt

    rp = np.array([0, 2, 2, 5])
    keys = np.array([7, 2**32 - 1, 0, 123456789, 99], dtype=np.uint64)
    binfmt.write(str(tmp_path / "c.xfb"), np.array([1, 0, 1]), rp, keys, np.arange(5))
    binfmt.write(str(tmp_path / "w.xfb"), np.array([1, 0, 1]), rp, keys, np.arange(5),
                 compact=False)
    c, w = binfmt.Shard(str(tmp_path / "c.xfb")), binfmt.Shard(str(tmp_path / "w.xfb"))
    assert c.compact and not w.compact and c.keys.dtype == np.uint32
    np.testing.assert_array_equal(c.keys.astype(np.uint64), w.keys)
    np.testing.assert_array_equal(c.fgid, w.fgid)
    assert os.path.getsize(tmp_path / "c.xfb") < os.path.getsize(tmp_path / "w.xfb")
    with pytest.raises(ValueError):
        binfmt.write(str(tmp_path / "x.xfb"), np.array([1]), np.array([0, 1]),
                     np.array([2**32], dtype=np.uint64), compact=True)


@pytest.mark.parametrize("kind,csr", [("lr", False), ("fm", False), ("lr", True)])
def test_compact_xfb_trains_like_wide(tmp_path, kind, csr):
    """A compact-key shard (u32 keys widened by the engine: in the
    field-major transpose, or by widen_keys for CSR blocks) trains exactly
    like the same shard stored with u64 keys."""
    (tmp_path / "c").mkdir()
    (tmp_path / "w").mkdir()
    _fixed_width_shards(tmp_path / "c", hash32=True, csr=csr)
    _fixed_width_shards(tmp_path / "w", hash32=True, compact="off", csr=csr)
    from xflow_amd.data import binfmt

    assert binfmt.Shard(str(tmp_path / "c" / "tr-00000.xfb")).compact
    a = _train_preds(tmp_path / "c", "p", kind=kind)
    b = _train_preds(tmp_path / "w", "p", kind=kind)
    assert len(a) == 100
    np.testing.assert_array_equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("csr", [False, True])
def test_compact_xfb_gpu_streamed_equals_wide(gpu_device, tmp_path, csr):
    """GPU: compact keys go over the host link as int32 (BlockStream) and are
    widened on the device (k_field_major<u32, u64> / widen_keys); training
    equals the u64-key shard bit for bit."""
    (tmp_path / "c").mkdir()
    (tmp_path / "w").mkdir()
    _fixed_width_shards(tmp_path / "c", rows=3000, hash32=True, csr=csr)
    _fixed_width_shards(tmp_path / "w", rows=3000, hash32=True, compact="off", csr=csr)
    a = _train_preds(tmp_path / "c", "p", device="cuda", block_rows=512)
    b = _train_preds(tmp_path / "w", "p", device="cuda", block_rows=512)
    assert len(a) == 1000
    np.testing.assert_array_equal(a, b)


def test_packed_xfb_roundtrip_and_training(tmp_path):
    """Version-3 packed shards (per-field dictionaries as u8 / u16 codes,
    direct u32 / u64 keys otherwise) expand to exactly the rows written, on
    the CPU backend's unpack_block, and train bit-identically to the same
    rows from a v1 shard through the Trainer."""
    import torch

    from xflow_amd.config import EngineConfig, ModelConfig, OptimConfig, TrainConfig
    from xflow_amd.data import binfmt
    from xflow_amd.engine import Engine
    from xflow_amd.trainer import Trainer

    rng = np.random.default_rng(5)
    rows, F = 70000, 6
    keys = np.empty((rows, F), np.uint64)
    keys[:, 0] = rng.integers(0, 40, rows) * 1000003            # u8 dictionary
    keys[:, 1] = rng.integers(0, 5000, rows) + (1 << 40)        # u16 dictionary
    keys[:, 2] = rng.integers(0, 1 << 31, rows)                 # direct u32
    keys[:, 3] = rng.integers(1 << 40, 1 << 62, rows, dtype=np.uint64)  # direct u64
    keys[:, 4] = rng.integers(0, 256, rows) * 7919
    keys[:, 5] = rng.integers(0, 65536, rows) * 31 + 5
    labels = (rng.random(rows) < 0.3).astype(np.float32)
    info = binfmt.write_packed(str(tmp_path / "p-00000.xfb"), labels, keys, block_rows=16384)
    assert info["widths"] == [1, 2, 4, 8, 1, 2], info
    eng = Engine(ModelConfig(kind="mvm"), OptimConfig(),
                 EngineConfig(table_log2_cap=12, max_rows=16384, max_nnz=16384 * F))
    r = binfmt.open_reader(str(tmp_path / "p-00000.xfb"))
    ks, ls = [], []
    while True:
        b = r.next()
        if b is None:
            break
        B = eng.unpack_packed(torch.from_numpy(np.array(b["packed"])), b["rows"], b["shard"],
                              with_fgid=True)
        assert B.field_major and B.nnz_per_row == F
        assert (B.fgid.view(F, -1) == torch.arange(F, dtype=torch.int32).view(F, 1)).all()
        ks.append(B.keys.view(F, -1).t().numpy().view(np.uint64))
        ls.append(B.labels.numpy())
    assert np.array_equal(np.concatenate(ks), keys)
    assert np.array_equal(np.concatenate(ls), labels)
    # the same rows as a v1 shard train to the same table
    binfmt.write(str(tmp_path / "q-00000.xfb"), labels, np.arange(rows + 1) * F, keys.reshape(-1),
                 np.tile(np.arange(F, dtype=np.int32), rows), compact=False)
    tables = []
    for prefix in ("p", "q"):
        cfg = TrainConfig(train_prefix=str(tmp_path / prefix), test_prefix=str(tmp_path / prefix),
                          epochs=1, threads=4, block_rows=16384, write_pred=False,
                          model=ModelConfig(kind="lr"), engine=EngineConfig(table_log2_cap=20))
        t = Trainer(cfg, device=torch.device("cpu"))
        t.train_epochs(1)
        k, w = t.table.export_table()
        o = np.argsort(k)
        tables.append((k[o], w.reshape(len(k), -1)[o]))
        t.close()
    assert np.array_equal(tables[0][0], tables[1][0])
    assert np.array_equal(tables[0][1], tables[1][1])


@pytest.mark.gpu
def test_packed_xfb_unpack_on_gpu(gpu_device, tmp_path):
    """k_unpack_block (csrc/hip/kernels_layout.hip) expands every code width
    and dictionary mode to the written keys, labels and field ids."""
    import torch

    from xflow_amd.config import EngineConfig, ModelConfig, OptimConfig
    from xflow_amd.data import binfmt
    from xflow_amd.engine import Engine

    rng = np.random.default_rng(9)
    rows, F = 100000, 5
    keys = np.empty((rows, F), np.uint64)
    keys[:, 0] = rng.integers(0, 64, rows) * 77
    keys[:, 1] = rng.integers(0, 30000, rows) + (1 << 50)
    keys[:, 2] = rng.integers(0, 1 << 32, rows, dtype=np.uint64)
    keys[:, 3] = rng.integers(1 << 33, 1 << 63, rows, dtype=np.uint64)
    keys[:, 4] = rng.integers(0, 3, rows)
    labels = (rng.random(rows) < 0.25).astype(np.float32)
    info = binfmt.write_packed(str(tmp_path / "g.xfb"), labels, keys, block_rows=65536)
    assert info["widths"] == [1, 2, 4, 8, 1]
    eng = Engine(ModelConfig(kind="mvm"), OptimConfig(),
                 EngineConfig(table_log2_cap=12, max_rows=65536, max_nnz=65536 * F), device=gpu_device)
    r = binfmt.open_reader(str(tmp_path / "g.xfb"))
    ks, ls = [], []
    while True:
        b = r.next()
        if b is None:
            break
        B = eng.unpack_packed(torch.from_numpy(np.array(b["packed"])).to(gpu_device), b["rows"],
                              b["shard"], with_fgid=True)
        assert (B.fgid.view(F, -1).cpu() == torch.arange(F, dtype=torch.int32).view(F, 1)).all()
        ks.append(B.keys.view(F, -1).t().cpu().numpy().view(np.uint64))
        ls.append(B.labels.cpu().numpy())
    assert np.array_equal(np.concatenate(ks), keys)
    assert np.array_equal(np.concatenate(ls), labels)
