"""Dedup scratch (persistence, epoch stamps, device-side rebuild), synthetic
data generator, FTRL / sigmoid scalar recipes, on the CPU backend and (gpu
marker) on the gfx950 HIP backend."""
import math
import os

import numpy as np
import pytest
import torch

from helpers import random_csr, to_batch
from xflow_amd.config import EngineConfig, ModelConfig, OptimConfig
from xflow_amd.data.synth import SynthConfig, SyntheticCriteo, criteo_vocab
from xflow_amd.engine import Engine
from xflow_amd.testing import torch_ref

DEVICES = [pytest.param("cpu", id="cpu"), pytest.param("cuda", id="gpu", marks=pytest.mark.gpu)]


def _dev(name):
    return torch.device("cuda", 0) if name == "cuda" else torch.device("cpu")


@pytest.mark.parametrize("devname", DEVICES)
def test_dedup_unique_count_over_many_steps_with_rebuild(devname):
    dev = _dev(devname)
    # tiny scratch (factor 2.5 of 512 nnz -> 2048 slots, rebuild at 1024 claims)
    eng = Engine(ModelConfig(), OptimConfig(),
                 EngineConfig(table_log2_cap=16, max_rows=64, max_nnz=512), device=dev)
    seen = set()
    for step in range(40):
        k, rp, fg, lab = random_csr(64, 6, vocab=400 + 50 * step, seed=step)
        b = to_batch(k, rp, fg, lab, dev)
        eng.train_step(b)
        assert eng.n_unique() == len(np.unique(k)), step
        seen.update(k.tolist())
    assert eng.table_size() == len(seen)
    assert not eng.overflowed()


@pytest.mark.parametrize("devname", DEVICES)
def test_eval_does_not_insert(devname):
    dev = _dev(devname)
    eng = Engine(ModelConfig(kind="fm", v_dim=4), OptimConfig(),
                 EngineConfig(table_log2_cap=12, max_rows=64, max_nnz=1024), device=dev)
    k, rp, fg, lab = random_csr(64, 6, seed=3)
    p = eng.eval_step(to_batch(k, rp, fg, lab, dev))
    assert eng.table_size() == 0
    assert torch.isfinite(p).all() and p.shape == (64,)


@pytest.mark.parametrize("devname", DEVICES)
def test_synthetic_criteo_shape(devname):
    dev = _dev(devname)
    rows = 4096
    cfg = SynthConfig()
    eng = Engine(ModelConfig(kind="mvm", v_dim=4), OptimConfig(),
                 EngineConfig(table_log2_cap=16, max_rows=rows, max_nnz=rows * cfg.fields),
                 device=dev)
    gen = SyntheticCriteo(eng, rows, cfg)
    b = gen.alloc_batch()
    gen.next(out=b)
    assert b.field_major
    # field-major layout [field][row]; the row-major generator gives its transpose
    k = b.keys.cpu().numpy().reshape(cfg.fields, rows).T
    assert (k >= 0).all() and (k < cfg.hash_space).all()
    assert (b.fgid.cpu().numpy().reshape(cfg.fields, rows).T == np.arange(cfg.fields)).all()
    rm = SyntheticCriteo(eng, rows, SynthConfig(field_major=False))
    brm = rm.alloc_batch()
    rm.next(out=brm)
    assert not brm.field_major
    np.testing.assert_array_equal(brm.keys.cpu().numpy().reshape(rows, cfg.fields), k)
    assert torch.equal(brm.labels, b.labels)
    assert torch.equal(brm.to_field_major().keys, b.keys)
    # the engine's transpose (HIP: LDS-tiled kernel) == torch's
    fm = brm.to_field_major(eng)
    assert torch.equal(fm.keys, b.keys) and torch.equal(fm.fgid, b.fgid)
    y = b.labels.cpu().numpy()
    assert set(np.unique(y)) <= {0.0, 1.0} and 0.1 < y.mean() < 0.45
    # power-law: the 3-valued field has very few distinct keys, big fields many
    small = cfg.vocab.index(3)
    assert len(np.unique(k[:, small])) <= 3
    assert len(np.unique(k[:, 13])) > 500
    # counter based: same (seed, step) -> same batch, next step differs
    b2 = gen.alloc_batch()
    gen.step = 0
    gen.next(out=b2)
    assert torch.equal(b.keys, b2.keys)
    gen.next(out=b2)
    assert not torch.equal(b.keys, b2.keys)
    assert sum(criteo_vocab()) >= 999_000_000


@pytest.mark.gpu
def test_synthetic_gpu_equals_cpu():
    rows = 2048
    cfg = SynthConfig()
    out = []
    for dev in (torch.device("cpu"), torch.device("cuda", 0)):
        eng = Engine(ModelConfig(), OptimConfig(),
                     EngineConfig(table_log2_cap=12, max_rows=rows, max_nnz=rows * 39), device=dev)
        gen = SyntheticCriteo(eng, rows, cfg)
        b = gen.alloc_batch()
        gen.next(out=b)
        out.append((b.keys.cpu().numpy(), b.labels.cpu().numpy()))
    # keys: float recipe from IEEE basic operations only -> bit-identical
    np.testing.assert_array_equal(out[0][0], out[1][0])
    assert (out[0][1] == out[1][1]).mean() > 0.999   # labels: one libm exp per row


def test_sigmoid_reference_clamps(native):
    eng = Engine(ModelConfig(), OptimConfig(), EngineConfig(table_log2_cap=8, max_rows=8,
                                                            max_nnz=64))
    x = torch.tensor([-40.0, -30.5, -30.0, -1.0, 0.0, 0.7, 30.0, 30.5, 50.0])
    p = torch_ref.sigmoid_ref(x)
    assert p[0] == pytest.approx(1e-6) and p[1] == pytest.approx(1e-6)
    assert p[-1] == 1.0 and p[-2] == 1.0
    ex = math.pow(2.718281828, 0.7)
    assert p[5].item() == pytest.approx(ex / (1 + ex), rel=1e-7)


@pytest.mark.parametrize("devname", DEVICES)
def test_ftrl_single_key_closed_form(devname):
    """One key, explicit gradients: table state follows ftrl.h:58-74 -- bit for
    bit with the engine's recipe (its two divisions by alpha are products with
    float(1/alpha), common.h), and within 1e-6 of the reference's quotients."""
    dev = _dev(devname)
    eng = Engine(ModelConfig(), OptimConfig(), EngineConfig(table_log2_cap=8, max_rows=8,
                                                            max_nnz=64), device=dev)
    a, b, l1, l2 = np.float32(0.05), np.float32(1.0), np.float32(5e-5), np.float32(10.0)
    ia = np.float32(np.float32(1.0) / a)
    w = n = z = np.float32(0)
    wr = nr = zr = np.float32(0)  # the reference's float recipe, divisions as written
    for g in [0.3, -0.2, 1e-5, 0.7, -0.9]:
        g = np.float32(g)
        eng.push([12345], [g])
        nn = np.float32(n + g * g)
        z = np.float32(z + np.float32(g - np.float32(np.float32(np.sqrt(nn) - np.sqrt(n)) * ia) * w))
        n = nn
        if abs(z) <= l1:
            w = np.float32(0)
        else:
            tmpr = np.float32(z - l1) if z > 0 else np.float32(z + l1)
            w = np.float32(tmpr / np.float32(-1.0 * np.float32(np.float32(b + np.sqrt(n)) * ia + l2)))
        nnr = np.float32(nr + g * g)
        zr = np.float32(zr + np.float32(g - np.float32(np.float32(np.sqrt(nnr) - np.sqrt(nr)) / a) * wr))
        nr = nnr
        if abs(zr) <= l1:
            wr = np.float32(0)
        else:
            tmpr = np.float32(zr - l1) if zr > 0 else np.float32(zr + l1)
            wr = np.float32(tmpr / np.float32(-1.0 * np.float32(np.float32(b + np.sqrt(nr)) / a + l2)))
        got = eng.pull([12345])[0, 0]
        assert got == w
        assert got == pytest.approx(wr, rel=1e-6, abs=1e-9)


@pytest.mark.gpu
def test_adaptive_scratch_capacity_matches_cpu(gpu_device):
    """The GPU dedup scratch shrinks to kScratchHeadroom (4) x the batch's
    unique keys, and a surge of distinct keys larger than the active table
    spills into the rest of the allocation (ScratchView::ctl[4]) instead of
    dropping keys, then grows it (device-side rebuilds); training still equals
    the CPU backend's (fixed-capacity scratch) step for step."""
    rows, fields = 8192, 8
    engines = [Engine(ModelConfig(kind="lr"), OptimConfig(),
                      EngineConfig(table_log2_cap=20, max_rows=rows, max_nnz=rows * fields),
                      device=d) for d in (torch.device("cpu"), gpu_device)]
    caps = []
    allk = []
    for step in range(12):
        k, rp, fg, lab = random_csr(rows, fields, 400, seed=500 + step, variable=False)
        if step >= 6:  # small vocabularies, then a surge of ~63 K distinct keys
            rng = np.random.default_rng(step)
            pool = rng.integers(0, 1 << 62, size=2_000_000, dtype=np.int64).astype(np.uint64)
            k = pool[rng.integers(0, pool.size, size=k.size)]
        allk.append(k)
        for e in engines:
            e.train_step(to_batch(k, rp, fg, lab, e.device))
        caps.append(engines[1].scratch_capacity())
    alloc = 1
    while alloc < int(rows * fields * 2.5) + 1:
        alloc <<= 1
    assert min(caps[:6]) < alloc, caps          # shrank while batches were small
    assert caps[-1] > min(caps[:6]), caps       # grew again for the surge
    assert not engines[1].overflowed()
    keys = np.unique(np.concatenate(allk))
    np.testing.assert_allclose(engines[1].pull(keys), engines[0].pull(keys), rtol=1e-4,
                               atol=1e-6)


@pytest.mark.parametrize("devname", DEVICES)
def test_device_pipeline_trains_like_sequential(devname):
    """Side-stream generation (DevicePipeline) feeds exactly the batches of
    sequential generation: same table after a few steps."""
    dev = _dev(devname)
    rows = 4096

    def mk():
        return Engine(ModelConfig(), OptimConfig(),
                      EngineConfig(table_log2_cap=20, max_rows=rows, max_nnz=rows * 39),
                      device=dev)

    a, b = mk(), mk()
    pipe = SyntheticCriteo(a, rows).pipeline()
    gen = SyntheticCriteo(b, rows)
    buf = gen.alloc_batch()
    for _ in range(4):
        a.train_step(pipe.next())
        pipe.done()
        gen.next(out=buf)
        b.train_step(buf)
    keys, _ = b.export_table()
    assert a.table_size() == b.table_size() == len(keys)
    np.testing.assert_allclose(a.pull(keys), b.pull(keys), rtol=1e-5, atol=1e-7)


@pytest.mark.gpu
def test_field_major_synthetic_lr_matches_cpu(gpu_device):
    """The bench path: field-major synthetic LR batches through the GPU step
    (field-chunked dedup, column-aggregated backward, bucket reduction) train
    the same table as the CPU backend.  5000 rows: dedup chunks straddle field
    boundaries and the last workgroups are partial."""
    from xflow_amd.engine import Batch

    rows = 5000
    cpu, gpu = (Engine(ModelConfig(), OptimConfig(),
                       EngineConfig(table_log2_cap=22, max_rows=rows, max_nnz=rows * 39), device=d)
                for d in (torch.device("cpu"), gpu_device))
    gen = SyntheticCriteo(cpu, rows)
    buf = gen.alloc_batch()
    for _ in range(3):
        gen.next(out=buf)
        cpu.train_step(buf)
        gpu.train_step(Batch(keys=buf.keys.to(gpu_device), labels=buf.labels.to(gpu_device),
                             nnz_per_row=buf.nnz_per_row, field_major=True))
    keys, _ = cpu.export_table()
    assert gpu.table_size() == len(keys)
    np.testing.assert_allclose(gpu.pull(keys), cpu.pull(keys), rtol=1e-4, atol=1e-6)
    assert gpu.read_stats()["rows"] == cpu.read_stats()["rows"] == 3 * rows


@pytest.mark.gpu
@pytest.mark.parametrize("rows", [3000, 65536])
def test_field_major_synthetic_mvm_matches_cpu(gpu_device, rows):
    """MVM on the bench shape (field-major, 39 fields, one field per column)
    with O(1) latent init, so the field products and gradients are live: the
    GPU backward (the bucket-reduction path) trains the same table as the
    CPU backend."""
    from xflow_amd.engine import Batch

    m = ModelConfig(kind="mvm", v_dim=10)
    o = OptimConfig(v_init_scale=1.0)
    cpu, gpu = (Engine(m, o, EngineConfig(table_log2_cap=22, max_rows=rows, max_nnz=rows * 39),
                       device=d) for d in (torch.device("cpu"), gpu_device))
    gen = SyntheticCriteo(cpu, rows)
    buf = gen.alloc_batch()
    for _ in range(3):
        gen.next(out=buf)
        cpu.train_step(buf)
        gpu.train_step(Batch(keys=buf.keys.to(gpu_device), labels=buf.labels.to(gpu_device),
                             fgid=buf.fgid.to(gpu_device), nnz_per_row=buf.nnz_per_row,
                             field_major=True))
    keys, _ = cpu.export_table()
    assert gpu.table_size() == len(keys)
    want = cpu.pull(keys)
    assert np.abs(want).max() > 1e-2
    np.testing.assert_allclose(gpu.pull(keys), want, rtol=1e-3, atol=1e-5)
    a, b = gpu.read_stats(), cpu.read_stats()
    print("mvm rows", rows, "gpu ln_loss/row", a["ln_loss"] / a["rows"], "cpu", b["ln_loss"] / b["rows"])
    assert abs(a["ln_loss"] - b["ln_loss"]) <= 1e-4 * abs(b["ln_loss"])


@pytest.mark.parametrize("devname", DEVICES)
def test_stamp_epoch_wrap(devname):
    """The dedup scratch stamps are one byte: epochs cycle through 1..255 and
    the stamps are cleared at the wrap.  300 steps over recurring keys train
    like the CPU backend (reference) across the wrap."""
    dev = _dev(devname)
    rows, fields = 256, 8
    engines = [Engine(ModelConfig(kind="lr"), OptimConfig(),
                      EngineConfig(table_log2_cap=16, max_rows=rows, max_nnz=rows * fields),
                      device=d) for d in ([torch.device("cpu")] + ([dev] if dev.type == "cuda" else []))]
    allk = []
    for step in range(300):
        k, rp, fg, lab = random_csr(rows, fields, 300, seed=9000 + step, variable=False)
        allk.append(k)
        for e in engines:
            e.train_step(to_batch(k, rp, fg, lab, e.device))
    keys = np.unique(np.concatenate(allk))
    for e in engines:
        assert not e.overflowed()
    np.testing.assert_allclose(engines[-1].pull(keys), engines[0].pull(keys), rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("devname", DEVICES)
@pytest.mark.parametrize("rows,F", [(1000, 39), (64, 1), (130, 64), (7, 13)])
def test_engine_field_major_transpose(devname, rows, F):
    """Backend field_major ([rows][F] -> [F][rows], HIP: LDS tiles of 64 rows,
    partial last tile) equals torch's transpose for u64 keys and i32 fgid."""
    from xflow_amd.engine import Batch

    dev = _dev(devname)
    eng = Engine(ModelConfig(kind="mvm", v_dim=4), OptimConfig(),
                 EngineConfig(table_log2_cap=10, max_rows=rows, max_nnz=rows * F), device=dev)
    rng = np.random.default_rng(rows + F)
    keys = torch.from_numpy(rng.integers(0, 1 << 62, rows * F, dtype=np.int64)).to(dev)
    fg = torch.from_numpy(rng.integers(0, 1 << 30, rows * F, dtype=np.int32)).to(dev)
    b = Batch(keys=keys, labels=torch.zeros(rows, device=dev), fgid=fg, nnz_per_row=F)
    a, t = b.to_field_major(eng), b.to_field_major()
    assert torch.equal(a.keys, t.keys) and torch.equal(a.fgid, t.fgid) and a.field_major


def test_synth_small_fast_path_bit_identical(tmp_path):
    """synth_sample<true> (32-bit rank conversion and multiply-high, used by
    k_synth when hash_space < 2^32 and every vocab < 2^31) returns the same
    key and weight bits as the general 64-bit recipe the CPU backend runs."""
    import shutil
    import subprocess

    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("g++ not available")
    src = tmp_path / "t.cpp"
    src.write_text(r'''
#include <cstdio>
#include <cstring>
#include <initializer_list>
#include "xflow/synth.h"
using namespace xflow;
int main() {
  const u64 vocabs[] = {1, 2, 3, 25, 1000, 65536, 10000000, 400000000, (1ull << 31) - 1};
  const double ss[] = {0.6, 1.0, 1.05, 1.3};
  const u64 spaces[] = {1, 7, 1000000000ull, (1ull << 32) - 1};
  long bad = 0, n = 0;
  for (u64 V : vocabs) for (double s : ss) for (u64 hs : spaces) {
    for (u64 r = 0; r < 20000; ++r) {
      const u64 seed = fmix64(r * 0x9e3779b97f4a7c15ull + V + hs);
      for (int f = 0; f < 39; f += 7) {
        const SynthField F = synth_field(V, s, f);
        float w0, w1;
        const u64 k0 = synth_sample<false>(seed, f, F, hs, 0.3f, w0);
        const u64 k1 = synth_sample<true>(seed, f, F, hs, 0.3f, w1);
        ++n;
        if (k0 != k1 || memcmp(&w0, &w1, 4) != 0) ++bad;
      }
    }
  }
  for (u64 a : {0ull, 1ull, ~0ull, 0x8000000000000000ull, 0x123456789abcdefull})
    for (u64 b : {0ull, 1ull, 0xffffffffull, 1000000000ull})
      if (mulhi64_u32(a, (u32)b) != mulhi64(a, b)) ++bad;
  std::printf("%ld %ld\n", n, bad);
  return bad != 0;
}
''')
    exe = tmp_path / "t"
    inc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "csrc", "include")
    r = subprocess.run([cxx, "-O2", "-std=c++17", "-ffp-contract=off", "-I" + inc, str(src), "-o",
                        str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
