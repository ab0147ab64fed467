"""Python face of the native Engine: torch-tensor batches, streams, checks.

The native engine (csrc/engine/engine.cpp) owns the HBM hash table and all
per-step buffers; this wrapper only validates tensors and hands device
addresses over.  On a GPU it always runs the gfx950 HIP backend on torch's
current stream (so engine kernels, torch ops and RCCL collectives are ordered
on one queue); on CPU it runs the native C++ backend.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch

from xflow_amd import native
from xflow_amd.config import EngineConfig, ModelConfig, OptimConfig


@dataclass
class Batch:
    """A batch of torch tensors on the engine's device: CSR (row_ptr), or
    fixed-width rows stored row-major or field-major (``field_major``: keys
    and fgid laid out [nnz_per_row][rows], see csrc/include/xflow/types.h)."""

    keys: torch.Tensor                  # int64 [nnz] (u64 bit patterns)
    labels: torch.Tensor                # float32 [rows]
    row_ptr: Optional[torch.Tensor] = None   # int32 [rows+1]; None => fixed nnz/row
    fgid: Optional[torch.Tensor] = None      # int32 [nnz]
    nnz_per_row: int = 0
    slice_rows: int = 0                 # rows per slice (gradient normaliser); 0 => all rows
    field_major: bool = False

    @property
    def rows(self) -> int:
        return int(self.labels.numel())

    @property
    def nnz(self) -> int:
        return int(self.keys.numel())

    def view(self):
        n = native.load()
        v = n.BatchView()
        v.keys = self.keys.data_ptr()
        v.labels = self.labels.data_ptr()
        v.row_ptr = self.row_ptr.data_ptr() if self.row_ptr is not None else 0
        v.fgid = self.fgid.data_ptr() if self.fgid is not None else 0
        v.rows = self.rows
        v.nnz = self.nnz
        v.nnz_per_row = self.nnz_per_row
        v.slice_rows = self.slice_rows
        v.col_stride = self.rows if self.field_major else 0
        return v

    def check(self, device: torch.device) -> None:
        for name, t, dt in (("keys", self.keys, torch.int64), ("labels", self.labels, torch.float32),
                            ("row_ptr", self.row_ptr, torch.int32), ("fgid", self.fgid, torch.int32)):
            if t is None:
                continue
            if t.dtype != dt:
                raise TypeError(f"batch.{name} must be {dt}, got {t.dtype}")
            if t.device != device:
                raise ValueError(f"batch.{name} on {t.device}, engine on {device}")
            if not t.is_contiguous():
                raise ValueError(f"batch.{name} must be contiguous")
        if self.row_ptr is None:
            if self.nnz_per_row <= 0 or self.nnz != self.rows * self.nnz_per_row:
                raise ValueError("fixed-width batch needs nnz == rows * nnz_per_row")
        elif self.row_ptr.numel() != self.rows + 1:
            raise ValueError("row_ptr must have rows+1 entries")
        if self.field_major and self.row_ptr is not None:
            raise ValueError("field-major batches are fixed-width (no row_ptr)")

    def to_field_major(self, engine: "Engine | None" = None) -> "Batch":
        """The same fixed-width batch stored field-major.  With an engine, its
        backend transposes (HIP: an LDS-tiled kernel on the engine's stream,
        csrc/hip/kernels_layout.hip); otherwise torch does."""
        if self.field_major:
            return self
        if self.row_ptr is not None:
            raise ValueError("only fixed-width batches have a field-major form")
        F = self.nnz_per_row
        if engine is not None and F <= 64:
            def t(x, widen=False):
                if x is None:
                    return None
                y = (torch.empty(x.numel(), dtype=torch.int64, device=x.device) if widen
                     else torch.empty_like(x))
                engine._sync_stream()
                engine.native.field_major(x.data_ptr(), y.data_ptr(), self.rows, F,
                                          x.element_size(), widen)
                return y
        else:
            def t(x, widen=False):
                if x is None:
                    return None
                y = x.view(self.rows, F).t().contiguous().view(-1)
                return widen_keys(y) if widen else y
        # compact (u32) keys of an .xfb shard are widened in the same pass
        return Batch(keys=t(self.keys, self.keys.dtype == torch.int32), labels=self.labels,
                     fgid=t(self.fgid), nnz_per_row=F, slice_rows=self.slice_rows,
                     field_major=True)


def widen_keys(keys: torch.Tensor) -> torch.Tensor:
    """Engine keys (int64 u64 bit patterns) from compact u32 keys held in an
    int32 tensor (data/binfmt.py compact shards); int64 keys pass through."""
    if keys.dtype == torch.int64:
        return keys
    if keys.dtype != torch.int32:
        raise TypeError(f"keys must be int64 or compact int32, got {keys.dtype}")
    return keys.to(torch.int64) & 0xFFFFFFFF


def _device_index(device: torch.device) -> int:
    if device.type == "cpu":
        return -1
    if device.type != "cuda":
        raise ValueError(f"unsupported device {device}")
    return device.index if device.index is not None else torch.cuda.current_device()


class Engine:
    """One rank's sparse trainer state (hash-table shard + worker buffers)."""

    def __init__(self, model: ModelConfig | None = None, optim: OptimConfig | None = None,
                 engine: EngineConfig | None = None, device: str | torch.device = "cpu"):
        self.model = model or ModelConfig()
        self.optim = optim or OptimConfig()
        self.cfg = engine or EngineConfig()
        self.device = torch.device(device)
        if self.device.type == "cuda":
            native.require_hip()
            if self.device.index is None:
                self.device = torch.device("cuda", torch.cuda.current_device())
        n = native.load()
        self._e = n.Engine(self.model.native(), self.optim.native(),
                           table_log2_cap=self.cfg.table_log2_cap, max_rows=self.cfg.max_rows,
                           max_nnz=self.cfg.max_nnz, max_slices=self.cfg.max_slices,
                           sum_slices=self.cfg.sum_slices, scratch_factor=self.cfg.scratch_factor,
                           device=_device_index(self.device), table_grow=self.cfg.table_grow,
                           grow_load=self.cfg.grow_load, max_log2_cap=self.cfg.max_log2_cap,
                           monitor_lag=self.cfg.monitor_lag, owner_group=self.cfg.owner_group,
                           grow_start=self.cfg.grow_start, csr=self.cfg.csr)
        if self.is_gpu != (self.device.type == "cuda"):
            raise RuntimeError("native engine backend does not match the requested device")

    # ---- properties -------------------------------------------------------
    @property
    def native(self):
        return self._e

    @property
    def is_gpu(self) -> bool:
        return bool(self._e.is_gpu)

    @property
    def backend_name(self) -> str:
        return self._e.backend_name

    @property
    def pstride(self) -> int:
        return int(self._e.pstride)

    @property
    def grad_width(self) -> int:
        """Floats per (key, slice) in the multi-rank gradient exchange."""
        return int(self._e.grad_width)

    @property
    def value_width(self) -> int:
        """Floats per pulled value row (pull outputs / values exchange): pstride,
        or 4 for reference-math FM on the GPU ((w, sum v, sum v^2, 0))."""
        return int(self._e.value_width)

    @property
    def params_per_key(self) -> int:
        return int(self._e.P)

    def _sync_stream(self) -> None:
        if self.is_gpu:
            self._e.set_stream(torch.cuda.current_stream(self.device).cuda_stream)

    # ---- single rank --------------------------------------------------------
    def train_step(self, batch: Batch) -> None:
        batch.check(self.device)
        self._sync_stream()
        self._e.train_step(batch.view())

    def eval_step(self, batch: Batch, pctr: torch.Tensor | None = None) -> torch.Tensor:
        batch.check(self.device)
        if pctr is None:
            pctr = torch.empty(batch.rows, dtype=torch.float32, device=self.device)
        self._sync_stream()
        self._e.eval_step(batch.view(), pctr.data_ptr())
        return pctr

    def train_view(self, view) -> None:
        """Train on a native BatchView (e.g. engine-staged synthetic batch)."""
        self._sync_stream()
        self._e.train_step(view)

    def synth_batch(self, rows: int, vocab, zipf_s, hash_space: int, seed: int, step: int,
                    planted_scale: float = 0.3, planted_bias: float = -1.2, slice_rows: int = 0,
                    out: Batch | None = None, field_major: bool = False):
        """Generate a synthetic batch on the engine's device.

        Without ``out`` the batch lives in engine-owned staging memory and a
        native BatchView is returned; with ``out`` (a Batch of preallocated
        tensors) the generator writes into those tensors and ``out`` is returned.
        ``field_major`` stores keys/fgid [field][row] (same rows, same values).
        """
        self._sync_stream()
        kw = {}
        if out is not None:
            kw = dict(keys=out.keys.data_ptr(), labels=out.labels.data_ptr(),
                      fgid=out.fgid.data_ptr() if out.fgid is not None else 0)
        v = self._e.synth_batch(int(rows), [int(x) for x in vocab], [float(s) for s in zipf_s],
                                int(hash_space), int(seed), int(step), float(planted_scale),
                                float(planted_bias), int(slice_rows), field_major=bool(field_major),
                                **kw)
        if out is None:
            return v
        out.nnz_per_row = len(vocab)
        out.slice_rows = int(slice_rows)
        out.field_major = bool(field_major)
        return out

    def push(self, keys, grads) -> None:
        self._e.push_host(np.asarray(keys, dtype=np.uint64),
                          np.asarray(grads, dtype=np.float32).reshape(-1))

    def prefill(self, n: int, seed: int = 0x5eed) -> None:
        """Insert n synthetic keys that no batch touches (bit 62 set): a table
        at the occupancy a long run reaches (untimed benchmark setup)."""
        self._sync_stream()
        self._e.prefill(int(n), int(seed))

    def pull(self, keys) -> np.ndarray:
        k = np.asarray(keys, dtype=np.uint64)
        return self._e.pull_host(k).reshape(len(k), self.params_per_key)

    # ---- multi-rank phases (driven by parallel.sparse_a2a) ----------------------
    # wb: worker buffer set (0/1) holding a prepared batch's dedup state, so the
    # next batch can be prepared while the current one is still in flight.
    def w_prepare(self, batch: Batch, world: int, counts: torch.Tensor, send_keys: torch.Tensor,
                  wb: int = 0, seq: int = -1):
        """seq >= 0 (world > 1): counts are written encoded with the prepare
        sequence number (csrc/include/xflow/backend.h encode_count)."""
        batch.check(self.device)
        self._sync_stream()
        self._e.w_prepare(batch.view(), world, counts.data_ptr(), send_keys.data_ptr(), int(wb),
                          int(seq))

    def s_pull(self, recv_keys: torch.Tensor, n: int, out_vals: torch.Tensor,
               insert: bool = True, buf: int = 0, offsets=None, keep_weights: bool = False) -> None:
        """Owner pull of n received keys into out_vals ([n, value_width]);
        ``offsets`` (world+1 source boundaries) lets the GPU backend group the
        sources for a one-launch apply; ``keep_weights`` keeps the pulled
        per-parameter weights for an apply after other updates (async step)."""
        self._sync_stream()
        self._e.s_pull(recv_keys.data_ptr(), int(n), out_vals.data_ptr(), insert, int(buf),
                       [int(o) for o in offsets] if offsets is not None else [],
                       bool(keep_weights))

    def w_forward(self, batch: Batch, pulled: torch.Tensor, n_send: int,
                  pctr: torch.Tensor | None, wb: int = 0) -> None:
        self._sync_stream()
        self._e.w_forward(batch.view(), pulled.data_ptr(), int(n_send),
                          pctr.data_ptr() if pctr is not None else 0, int(wb))

    def w_forward_backward(self, batch: Batch, pulled: torch.Tensor, n_send: int,
                           grads_out: torch.Tensor, masks_out: torch.Tensor | None,
                           S: int = 0, wb: int = 0, group: int = 0) -> None:
        """S > SLICE_GROUP: slice group ``group`` of the step only (its rows;
        grads_out holds group_slices(S, group) slices per key)."""
        self._sync_stream()
        self._e.w_forward_backward(batch.view(), pulled.data_ptr(), int(n_send),
                                   grads_out.data_ptr(),
                                   masks_out.data_ptr() if masks_out is not None else 0, int(S),
                                   int(wb), int(group))

    def s_apply(self, recv_keys: torch.Tensor, recv_grads: torch.Tensor,
                recv_masks: torch.Tensor | None, offsets, S: int, buf: int = 0) -> None:
        self._sync_stream()
        self._e.s_apply(recv_keys.data_ptr(), recv_grads.data_ptr(),
                        recv_masks.data_ptr() if recv_masks is not None else 0,
                        [int(o) for o in offsets], int(S), int(buf))

    def w_finish(self) -> None:
        self._sync_stream()
        self._e.w_finish()

    # ---- stats / checkpoint -------------------------------------------------
    def slices_of(self, batch: Batch) -> int:
        return int(self._e.slices_of(batch.view()))

    @staticmethod
    def slice_groups(S: int) -> list[int]:
        """Slices of each slice group of an S-slice step (Engine::slice_groups:
        more than 32 slices run in groups of 32, each group >= 2 slices)."""
        from xflow_amd import native

        n = native.load()
        return [int(n.Engine.group_slices(int(S), g)) for g in range(int(n.Engine.slice_groups(int(S))))]

    def read_stats(self, reset: bool = False, which: int = 0) -> dict:
        self._sync_stream()
        return self._e.read_stats(reset, which)

    def table_size(self) -> int:
        self._sync_stream()
        return int(self._e.table_size())

    @property
    def layout(self) -> dict:
        """Table slot layout (model kind, params per key, optimizer, words per slot)."""
        return dict(self._e.layout)

    @property
    def table_capacity(self) -> int:
        """Slots of this rank's table shard (grows, see EngineConfig.table_grow)."""
        return int(self._e.table_capacity)

    @property
    def table_growths(self) -> int:
        """Times the table grew (each: one or more segment splits)."""
        return int(self._e.table_growths)

    @property
    def csr_steps(self) -> int:
        """Steps of several slices that ran on the CSR path (one reduction and
        one apply of only the touched (key, slice) pairs, Engine::train_step_csr)."""
        return int(self._e.csr_steps)

    @property
    def table_splits(self) -> int:
        """Segments split so far (each added one segment of memory)."""
        return int(self._e.table_splits)

    @property
    def table_geometry(self) -> dict:
        """{seg_log2, level, split, segments} (TableView, csrc/include/xflow/backend.h)."""
        g, lv, sp, ns = self._e.table_geometry
        return {"seg_log2": int(g), "level": int(lv), "split": int(sp), "segments": int(ns)}

    @property
    def table_committed(self) -> int:
        """Device bytes committed to the table's address range."""
        return int(self._e.table_committed)

    @property
    def grow_seconds(self) -> float:
        """Host seconds spent in growth calls (memory mapping + split launches)."""
        return float(self._e.grow_seconds)

    @property
    def monitor_waits(self) -> int:
        """Host waits of the capacity monitor (bounded run-ahead, exact-size reads)."""
        return int(self._e.monitor_waits)

    def parse_text(self, text: torch.Tensor, n: int, out: dict, row_mod: int = 1):
        """libffm bytes text[:n] (uint8, engine device, 16-byte aligned,
        allocated >= n + 32 bytes) ->
        out["keys"/"fgid"/"row_ptr"/"labels"] on the device (kernels_parse.hip;
        reader.cpp's rules).  Returns (rows, occurrences, shortest row,
        longest row, occurrences of the first rows - rows % row_mod rows)."""
        self._sync_stream()
        if text.numel() < n + 32 and text.is_cuda:
            raise ValueError("parse_text: the text tensor needs >= n + 32 bytes")
        return tuple(int(x) for x in self._e.parse_text(
            text.data_ptr(), int(n), out["keys"].data_ptr(), out["fgid"].data_ptr(),
            out["row_ptr"].data_ptr(), out["labels"].data_ptr(), int(out["labels"].numel()),
            int(out["keys"].numel()), int(row_mod)))

    def unpack_packed(self, block: torch.Tensor, rows: int, shard, slice_rows: int = 0,
                      with_fgid: bool = False, used: int = -1) -> Batch:
        """A packed (version 3) .xfb block -- its raw bytes as a uint8 tensor
        on this engine's device -- as a field-major Batch (keys expanded from
        the per-field codes / dictionaries on the device, Backend::unpack_block).
        used >= 0: only the first `used` rows (the slicing rule's remainder drop)."""
        if block.device != self.device or block.dtype != torch.uint8:
            raise ValueError("unpack_packed: uint8 block bytes on the engine's device")
        F = shard.F
        dd = shard.device_dicts(self.device)
        keys = torch.empty(F * rows, dtype=torch.int64, device=self.device)
        labels = torch.empty(rows, dtype=torch.float32, device=self.device)
        fgid = torch.empty(F * rows, dtype=torch.int32, device=self.device) if with_fgid else None
        cols = shard.columns(rows)
        if block.numel() < cols[-1] + rows * shard.widths[-1]:
            raise ValueError("unpack_packed: block shorter than its columns")
        self._sync_stream()
        self._e.unpack_block(block.data_ptr(), int(rows), list(shard.widths), [int(c) for c in cols],
                             [dd[f] for f in range(F)], list(shard.fgid_cols), keys.data_ptr(),
                             labels.data_ptr(), fgid.data_ptr() if fgid is not None else 0)
        if 0 <= used < rows:  # (field-major: each field's first `used` rows)
            keys = keys.view(F, rows)[:, :used].contiguous().view(-1)
            labels = labels[:used]
            if fgid is not None:
                fgid = fgid.view(F, rows)[:, :used].contiguous().view(-1)
        return Batch(keys=keys, labels=labels, fgid=fgid, nnz_per_row=F, slice_rows=slice_rows,
                     field_major=True)

    def count_records(self, on: bool = True) -> None:
        """Count the gradient-reduction records the producers write."""
        self._e.count_records(bool(on))

    def take_records(self) -> int:
        """Records written since the last call (-1: never counted)."""
        self._sync_stream()
        return int(self._e.take_records())

    @property
    def monitor_wait_seconds(self) -> float:
        """Host seconds blocked by the monitor's run-ahead bound."""
        return float(self._e.monitor_wait_seconds)

    def grow_table(self, log2_cap: int) -> None:
        """Grow the table to >= 2^log2_cap slots now by segment splits (normally
        automatic)."""
        self._sync_stream()
        self._e.grow_table(int(log2_cap))

    def end_step(self) -> None:
        """Queue the step's capacity snapshot (the sharded steps call it via
        w_finish; raises if an earlier step overflowed)."""
        self._sync_stream()
        self._e.end_step()

    def n_unique(self) -> int:
        self._sync_stream()
        return int(self._e.n_unique())

    def scratch_capacity(self) -> int:
        """Active dedup scratch capacity (device-adaptive on the GPU)."""
        self._sync_stream()
        return int(self._e.scratch_capacity())

    def overflowed(self) -> bool:
        self._sync_stream()
        return bool(self._e.overflowed())

    def nonzero_weights(self) -> int:
        """Exactly non-zero (key, param) weights in this shard (L1 sparsity)."""
        self._sync_stream()
        return int(self._e.nonzero_weights())

    def download_small(self, dst: torch.Tensor, src: torch.Tensor) -> None:
        """Queue a copy of a small device tensor into pinned host memory on the
        current stream without the copy engine (read it after an event
        recorded behind this call)."""
        if self.is_gpu and not dst.is_pinned():
            raise ValueError("download_small: dst must be pinned host memory")
        if dst.numel() * dst.element_size() < src.numel() * src.element_size():
            raise ValueError("download_small: dst too small")
        self._sync_stream()
        self._e.download_small(dst.data_ptr(), src.contiguous().data_ptr(),
                               src.numel() * src.element_size())

    def eval_metrics(self, pctr: torch.Tensor, labels: torch.Tensor) -> dict:
        """AUC / logloss of predictions on this engine's device, computed there
        (GPU: radix sort + rank sums; only scalars come back).  Returns the
        reference's printed line (base.h:84-110) with auc / logloss_printed /
        ln_logloss / n / tp."""
        if pctr.device != self.device or labels.device != self.device:
            raise ValueError("eval_metrics: tensors must be on the engine's device")
        p = pctr.contiguous().float()
        y = labels.contiguous().float()
        if p.numel() != y.numel():
            raise ValueError("eval_metrics: pctr and labels differ in length")
        self._sync_stream()
        return dict(self._e.eval_metrics(p.data_ptr(), y.data_ptr(), int(p.numel())))

    def export_table(self):
        self._sync_stream()
        return self._e.export_table()

    def import_table(self, keys: np.ndarray, words: np.ndarray) -> None:
        self._sync_stream()
        self._e.import_table(np.ascontiguousarray(keys, dtype=np.uint64),
                             np.ascontiguousarray(words, dtype=np.uint32))

    @property
    def state_words(self) -> int:
        return int(self._e.state_words)

    def save(self, path: str) -> None:
        self._sync_stream()
        self._e.save(path)

    def load(self, path: str) -> None:
        self._sync_stream()
        self._e.load(path)

    def synchronize(self) -> None:
        self._e.synchronize()
