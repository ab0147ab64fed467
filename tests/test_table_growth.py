"""Parameter-table capacity management (the reference's store is an unbounded
unordered_map, /root/reference/src/optimizer/ftrl.h:54-56,84).

* A table that starts small grows (segment splits, linear hashing over the
  table's segments: TableView in csrc/include/xflow/backend.h) before its
  load passes grow_load, and the trained model is bitwise the one of a
  pre-sized table.
* Splits of a populated table -- partial levels, wrapped clusters -- keep
  every key and its state words, and lookups find them.
* Growth queues device work only: a rank that grows in the middle of a
  lock-step multi-rank run makes no host sync (its peers wait for nothing
  but the split kernels).
* A fixed table that fills up fails within monitor_lag steps, not at epoch
  end.
* Growth in the middle of a staleness-k step re-probes the slots of the
  pulled-but-not-yet-applied server buffers.
"""
import os

import numpy as np
import pytest
import torch

from dist_utils import run_world
from helpers import to_batch
from xflow_amd.config import EngineConfig, ModelConfig, OptimConfig
from xflow_amd.engine import Engine

DEVICES = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]


def _dev(name):
    if name == "cuda":
        if not torch.cuda.is_available():
            pytest.fail("gpu test selected but torch sees no GPU")
        return torch.device("cuda", 0)
    return torch.device("cpu")


def _fresh_csr(rows, fields, seed, reuse=0.5):
    """Fixed-width rows; about `reuse` of the occurrences draw from a small
    recurring pool, the rest are new keys (the table fills quickly)."""
    rng = np.random.default_rng(seed)
    pool = rng.integers(1, 1 << 62, size=fields * rows, dtype=np.int64)
    hot = (np.arange(500, dtype=np.int64) * 0x9E3779B97F4A7C1 + 12345) % (1 << 62)
    keys = np.where(rng.random(rows * fields) < reuse, hot[rng.integers(0, 500, rows * fields)],
                    pool).astype(np.uint64)
    rp = (np.arange(rows + 1) * fields).astype(np.int32)
    fg = np.tile(np.arange(fields, dtype=np.int32), rows)
    lab = (rng.random(rows) < 0.3).astype(np.float32)
    return keys, rp, fg, lab


def _train(dev, kind, log2_cap, steps=14, rows=2048, grow=True, lag=2):
    e = Engine(ModelConfig(kind=kind, v_dim=4), OptimConfig(),
               EngineConfig(table_log2_cap=log2_cap, max_rows=rows, max_nnz=rows * 12,
                            table_grow=grow, monitor_lag=lag), device=dev)
    allk = []
    for step in range(steps):
        k, rp, fg, lab = _fresh_csr(rows, 8, seed=77 + step)
        allk.append(k)
        e.train_step(to_batch(k, rp, fg, lab, dev))
    return e, np.unique(np.concatenate(allk))


@pytest.mark.parametrize("devname", DEVICES)
@pytest.mark.parametrize("kind", ["lr", "fm"])
def test_growth_equals_presized_table(devname, kind):
    dev = _dev(devname)
    small, keys = _train(dev, kind, 16)
    big, _ = _train(dev, kind, 20)
    assert small.table_growths >= 1 and big.table_growths == 0
    assert small.table_capacity > 1 << 16
    n = small.table_size()
    assert n == big.table_size() == len(keys)
    # the small table went past 0.9 of its original capacity
    assert n > 0.9 * (1 << 16)
    assert n <= 0.8 * small.table_capacity  # (kept below grow_load)
    assert not small.overflowed()
    a, b = small.pull(keys), big.pull(keys)
    np.testing.assert_array_equal(a.view(np.uint32), b.view(np.uint32))


@pytest.mark.parametrize("devname", DEVICES)
def test_fixed_table_overflow_fails_within_lag(devname):
    dev = _dev(devname)
    lag = 1
    e = Engine(ModelConfig(kind="lr"), OptimConfig(),
               EngineConfig(table_log2_cap=12, max_rows=2048, max_nnz=2048 * 12, table_grow=False,
                            monitor_lag=lag), device=dev)
    failed_at = None
    first_full = None
    for step in range(12):
        k, rp, fg, lab = _fresh_csr(2048, 8, seed=5 + step)
        try:
            e.train_step(to_batch(k, rp, fg, lab, dev))
        except RuntimeError as ex:
            assert "overflow" in str(ex)
            failed_at = step
            break
        if first_full is None and e.overflowed():  # (syncs: the step has run)
            first_full = step
    assert failed_at is not None, "a full fixed table never raised"
    # the overflowing step is the first one (4096 slots, ~15 K keys per step);
    # the raise comes at most lag + 1 step calls later
    assert first_full == 0 or first_full is None
    assert failed_at <= 1 + lag


def _async_growth_worker(rank, world, out_dir, log2_cap):
    from xflow_amd.parallel.async_p2p import AsyncShardedEngine

    eng = Engine(ModelConfig(kind="fm", v_dim=4), OptimConfig(),
                 EngineConfig(table_log2_cap=log2_cap, max_rows=256, max_nnz=256 * 12))
    sh = AsyncShardedEngine(eng, staleness=2)
    for step in range(8):
        k, rp, fg, lab = _fresh_csr(256, 8, seed=100 * step + rank)
        sh.train_step(to_batch(k, rp, fg, lab, torch.device("cpu")), S=1)
    sh.flush()
    keys, _ = eng.export_table()
    np.save(os.path.join(out_dir, f"k{rank}_{log2_cap}.npy"), keys)
    np.save(os.path.join(out_dir, f"v{rank}_{log2_cap}.npy"), eng.pull(keys))
    np.save(os.path.join(out_dir, f"g{rank}_{log2_cap}.npy"), np.array([eng.table_growths]))


def test_growth_with_pending_staleness_buffers(tmp_path):
    """gloo, 2 ranks, staleness 2: tables of 2^10 slots grow while two steps'
    pushes are pending; the result equals 2^16-slot tables bit for bit."""
    for cap in (10, 16):
        run_world(_async_growth_worker, 2, str(tmp_path), cap)
    grew = sum(int(np.load(tmp_path / f"g{r}_10.npy")[0]) for r in range(2))
    assert grew >= 2
    for r in range(2):
        ka, kb = np.load(tmp_path / f"k{r}_10.npy"), np.load(tmp_path / f"k{r}_16.npy")
        oa, ob = np.argsort(ka), np.argsort(kb)
        np.testing.assert_array_equal(ka[oa], kb[ob])
        va, vb = np.load(tmp_path / f"v{r}_10.npy"), np.load(tmp_path / f"v{r}_16.npy")
        np.testing.assert_array_equal(va[oa].view(np.uint32), vb[ob].view(np.uint32))


@pytest.mark.parametrize("devname", DEVICES)
def test_diverged_model_is_flagged(devname):
    """A non-finite weight makes the forward's predictions non-finite: the
    values are clamped before the fixed-point gradient sums (no undefined
    conversion) and the capacity monitor raises within monitor_lag steps."""
    dev = _dev(devname)
    e = Engine(ModelConfig(kind="lr"), OptimConfig(),
               EngineConfig(table_log2_cap=16, max_rows=512, max_nnz=512 * 12, monitor_lag=1),
               device=dev)
    k, rp, fg, lab = _fresh_csr(512, 8, seed=3, reuse=0.9)
    e.train_step(to_batch(k, rp, fg, lab, dev))
    e.push(np.unique(k)[:50], np.full(50, np.nan, np.float32))  # poison some weights
    with pytest.raises(RuntimeError, match="non-finite"):
        for _ in range(4):
            e.train_step(to_batch(k, rp, fg, lab, dev))
    assert e.overflowed()


def _rand_state(rng, n, words):
    keys = np.unique(rng.integers(1, 1 << 62, size=n + n // 8, dtype=np.int64))[:n]
    rng.shuffle(keys)
    w = rng.integers(0, 1 << 20, size=(len(keys), words), dtype=np.int64).astype(np.uint32)
    # state words as small positive floats (valid n / z accumulators)
    w = (w.astype(np.float32) / (1 << 16)).view(np.uint32)
    return keys.astype(np.uint64), w


@pytest.mark.parametrize("devname", DEVICES)
@pytest.mark.parametrize("kind", ["lr", "fm"])
def test_segment_splits_keep_every_key(devname, kind):
    """Chunks of imported (key, state) rows into a 2^12-slot table (one
    segment): each chunk's guard splits segments of a populated table, level
    after level and part-way through levels; after every chunk the export is
    exactly the imported rows and every key's pulled weights equal those of
    a pre-sized table holding the same rows."""
    dev = _dev(devname)
    mk = lambda cap: Engine(ModelConfig(kind=kind, v_dim=4), OptimConfig(),
                            EngineConfig(table_log2_cap=cap, max_rows=256, max_nnz=4096), device=dev)
    e, big = mk(12), mk(18)
    rng = np.random.default_rng(11)
    keys, words = _rand_state(rng, 40000, e.state_words)
    done = 0
    geoms = set()
    for chunk in [2000, 1000, 500, 500, 1500, 3000, 3500, 8000, 20000]:
        e.import_table(keys[done:done + chunk], words[done:done + chunk])
        big.import_table(keys[done:done + chunk], words[done:done + chunk])
        done += chunk
        g = e.table_geometry
        geoms.add((g["level"], g["split"]))
        assert e.table_capacity == g["segments"] << g["seg_log2"]
        assert e.table_size() == done and not e.overflowed()
        ek, ew = e.export_table()
        ew = ew.reshape(len(ek), -1)
        o = np.argsort(ek)
        ref = np.argsort(keys[:done])
        np.testing.assert_array_equal(ek[o], keys[:done][ref])
        np.testing.assert_array_equal(ew[o], words[:done][ref])
        q = keys[:done]
        np.testing.assert_array_equal(e.pull(q).view(np.uint32), big.pull(q).view(np.uint32))
    assert e.table_splits >= 8 and e.table_growths >= 4
    # some chunk ended part-way through a level (split != 0)
    assert any(sp for _, sp in geoms)
    assert done <= 0.8 * e.table_capacity


def _sync_growth_worker(rank, world, out_dir, caps):
    from xflow_amd.parallel.sparse_a2a import ShardedEngine

    cap = caps[rank]
    eng = Engine(ModelConfig(kind="fm", v_dim=4), OptimConfig(),
                 EngineConfig(table_log2_cap=cap, max_rows=256, max_nnz=256 * 12))
    sh = ShardedEngine(eng)
    for step in range(10):
        k, rp, fg, lab = _fresh_csr(256, 8, seed=300 * step + rank)
        sh.train_step(to_batch(k, rp, fg, lab, torch.device("cpu")), S=1)
    keys, _ = eng.export_table()
    tag = "-".join(map(str, caps))
    np.save(os.path.join(out_dir, f"k{rank}_{tag}.npy"), keys)
    np.save(os.path.join(out_dir, f"v{rank}_{tag}.npy"), eng.pull(keys))
    np.save(os.path.join(out_dir, f"g{rank}_{tag}.npy"),
            np.array([eng.table_growths, eng.monitor_waits, eng.table_splits]))


def test_one_rank_grows_mid_run_without_host_sync(tmp_path):
    """gloo, 2 lock-step ranks: rank 0's shard starts at 2^10 slots and grows
    several times mid-run, rank 1's is pre-sized.  The growing rank makes no
    host wait for it (monitor_waits == 0: the split is queued device work),
    and both shards equal a run where both are pre-sized, bit for bit."""
    run_world(_sync_growth_worker, 2, str(tmp_path), (10, 16))
    run_world(_sync_growth_worker, 2, str(tmp_path), (16, 16))
    g0 = np.load(tmp_path / "g0_10-16.npy")
    assert g0[0] >= 2 and g0[2] >= 2 and g0[1] == 0
    for r in range(2):
        ka, kb = np.load(tmp_path / f"k{r}_10-16.npy"), np.load(tmp_path / f"k{r}_16-16.npy")
        oa, ob = np.argsort(ka), np.argsort(kb)
        np.testing.assert_array_equal(ka[oa], kb[ob])
        va, vb = np.load(tmp_path / f"v{r}_10-16.npy"), np.load(tmp_path / f"v{r}_16-16.npy")
        np.testing.assert_array_equal(va[oa].view(np.uint32), vb[ob].view(np.uint32))
