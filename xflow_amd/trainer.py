"""Multi-rank training loop over libffm shards (Python orchestration of the
native engine).

Reference: the workers' batch_training / predict / train
(/root/reference/src/model/lr/lr_worker.cc:73-217, fm_worker.cc:98-287,
mvm_worker.cc:109-314).  Same data contract: rank r trains on
``<train_prefix>-%05d`` (r) block by block (2 MB blocks, rows split into
``threads`` slices of rows//threads, remainder dropped), then rank 0 predicts
``<test_prefix>-00000``, writes ``pred_0_0.txt`` and prints the reference's
``logloss: .. auc = ..`` line.

Differences by design (MI355X-first):
* the parameter server is the ranks' own HBM table shards; Pull/Push are the
  sparse all-to-alls of parallel/sparse_a2a.py (world > 1) or the fused
  single-rank step;
* the reference's Hogwild threads become the S slices of one step (all read
  the same weights, pushes applied in slice order), or one step per slice
  (serial_slices);
* ranks advance in lock-step; a rank that ran out of blocks joins each
  exchange with an empty batch until every rank is done with the epoch.  The
  multi-rank loop is pipelined (each step prepares the rank's next batch) and
  learns that the epoch is over from the counts exchange it does anyway (a
  source without data sends -1 counts, ShardedEngine.train_step) -- no
  per-block collective or host synchronisation.
"""
from __future__ import annotations

import os
import warnings
import sys
import time
from typing import Optional

import numpy as np
import torch

from xflow_amd import checkpoint
from xflow_amd import native as _native
from xflow_amd.config import TrainConfig, model_kind
from xflow_amd.data import binfmt
from xflow_amd.data.textstream import TextStream
from xflow_amd.data.upload import BlockStream
from xflow_amd.engine import Batch, Engine, widen_keys
from xflow_amd.metrics import MetricsLogger, reference_auc
from xflow_amd.parallel import dist as xdist
from xflow_amd.testing.hashing import owner_of
from xflow_amd.utils.faults import injector_from_env, watchdog_from_env
from xflow_amd.utils.trace import PhaseTimer, StreamTimeline


def shard_path(prefix: str, rank: int) -> str:
    return "%s-%05d" % (prefix, rank)


def _say(msg: str) -> None:
    print(msg, flush=True)


def _uniform_width(row_ptr) -> int:
    """Features per row when every row has the same (non-zero) count, else 0."""
    lens = np.diff(np.asarray(row_ptr))
    if len(lens) == 0 or lens[0] <= 0 or not np.all(lens == lens[0]):
        return 0
    return int(lens[0])


class Trainer:
    def __init__(self, cfg: TrainConfig, device: Optional[torch.device] = None):
        self.cfg = cfg
        self.world = xdist.start(device)
        self.rank = xdist.my_rank()
        self.device = device or xdist.device_for_rank()
        self.threads = cfg.resolved_threads()
        self.concurrent = not cfg.serial_slices
        # any thread count: beyond 32 slices a step runs its slices in groups
        # of 32 over one pull (Engine.slice_groups), the same semantics
        self.S = self.threads if self.concurrent else 1
        max_block = max(cfg.train_block_bytes, cfg.resolved_test_block())
        ecfg = cfg.engine
        ecfg.max_rows = max(ecfg.max_rows, max_block // 2 + 16)
        ecfg.max_nnz = max(ecfg.max_nnz, max_block // 2 + 16)
        # binary shards (.xfb) come in blocks of block_rows rows: size for the largest
        self.block_rows = cfg.block_rows or 65536
        for p in (shard_path(cfg.train_prefix, xdist.my_rank()), shard_path(cfg.test_prefix, 0)):
            xfb = binfmt.shard_file(p)
            if xfb:
                rows, nnz = binfmt.max_block(xfb, self.block_rows)
                ecfg.max_rows = max(ecfg.max_rows, rows)
                ecfg.max_nnz = max(ecfg.max_nnz, nnz)
        ecfg.max_slices = max(ecfg.max_slices, self.S)
        self.sharded = None
        self.aps = None
        if self.world > 1 and cfg.async_ps:
            # the asynchronous parameter server: this rank's table shard lives
            # in the server engine (its thread's), batches and forward passes
            # in the worker engine; served between epochs only when paused
            from xflow_amd.parallel.async_ps import AsyncParameterServer

            self.aps = AsyncParameterServer(cfg.model, cfg.optim, ecfg, self.device,
                                            staleness=cfg.staleness, slices=self.S, start=False,
                                            slow_ms=0)  # (slow_rank: the injector sleeps)
            self.engine = self.aps.worker
            self.table = self.aps.server
        else:
            self.engine = Engine(cfg.model, cfg.optim, ecfg, device=self.device)
            # the engine holding this rank's table shard
            self.table = self.engine
        if self.aps is not None:
            pass
        elif self.world > 1 and cfg.async_p2p:
            from xflow_amd.parallel.async_p2p import AsyncShardedEngine

            self.sharded = AsyncShardedEngine(self.engine, staleness=cfg.staleness)
        elif self.world > 1:
            from xflow_amd.parallel.sparse_a2a import ShardedEngine

            self.sharded = ShardedEngine(self.engine)
        self.metrics = MetricsLogger(cfg.metrics_file, self.rank)
        self.timer = PhaseTimer(self.device, enabled=bool(os.environ.get("XFLOW_TRACE")))
        self.watchdog = watchdog_from_env(f"xflow-rank{self.rank}")
        self.faults = injector_from_env(self.rank)
        self.epoch = 0
        self.steps = 0
        self.samples = 0
        self.resumed = False
        self._with_fgid = model_kind(cfg.model.kind) == 2
        self._resident = None

    # ------------------------------------------------------------------ data
    def _to_batch(self, blk: Optional[dict], used: int, slice_rows: int) -> Batch:
        dev = self.device
        if blk is not None and used > 0 and "packed" in blk:
            # a packed (v3 .xfb) block: its bytes, expanded on the device
            p = blk["packed"]
            if not isinstance(p, torch.Tensor):
                p = torch.from_numpy(np.array(p)).to(dev)
            return self.engine.unpack_packed(p, int(blk["rows"]), blk["shard"], slice_rows,
                                             self._with_fgid, used)
        if blk is not None and used > 0 and isinstance(blk["keys"], torch.Tensor):
            return self._device_batch(blk, used, slice_rows)
        if blk is None or used <= 0:
            return Batch(keys=torch.empty(0, dtype=torch.int64, device=dev),
                         labels=torch.empty(0, dtype=torch.float32, device=dev),
                         row_ptr=torch.zeros(1, dtype=torch.int32, device=dev),
                         fgid=torch.empty(0, dtype=torch.int32, device=dev),
                         slice_rows=max(slice_rows, 1))
        rp = blk["row_ptr"][: used + 1]
        nnz = int(rp[-1])
        pin = dev.type == "cuda"

        def up(a):
            with warnings.catch_warnings():  # read-only .xfb mappings: only ever read
                warnings.simplefilter("ignore", UserWarning)
                t = torch.from_numpy(np.ascontiguousarray(a))
            if pin:
                t = t.pin_memory()
            return t.to(dev, non_blocking=True)

        F = _uniform_width(rp) if self.cfg.fixed_width else 0
        k = np.asarray(blk["keys"][:nnz])
        # (compact u32 .xfb keys upload as int32 and widen on the device)
        keys = up(k.view(np.int32) if k.dtype == np.uint32 else k.view(np.int64))
        fgid = up(blk["fgid"][:nnz]) if self._with_fgid else None
        if F:
            return Batch(keys=keys, labels=up(blk["labels"][:used]), fgid=fgid, nnz_per_row=F,
                         slice_rows=slice_rows).to_field_major(self.engine)
        return Batch(keys=widen_keys(keys), labels=up(blk["labels"][:used]), row_ptr=up(rp),
                     fgid=fgid, slice_rows=slice_rows)

    def _device_batch(self, blk: dict, used: int, slice_rows: int) -> Batch:
        """Batch over a block already on the device (data.upload.BlockStream,
        or data.textstream.TextStream: its parse counted the used rows' nnz)."""
        if "row_ptr_host" in blk:
            nnz = int(blk["row_ptr_host"][used])
        else:
            if used != blk["rows"] - blk["rows"] % (1 if self.cfg.keep_remainder else self.threads):
                raise ValueError("text-stream block: used rows differ from the parse's")
            nnz = int(blk["nnz_used"])
        fgid = blk["fgid"][:nnz] if self._with_fgid else None
        F = blk["nnz_per_row"] if self.cfg.fixed_width else 0
        if F:
            return Batch(keys=blk["keys"][:nnz], labels=blk["labels"][:used], fgid=fgid,
                         nnz_per_row=F, slice_rows=slice_rows).to_field_major(self.engine)
        return Batch(keys=widen_keys(blk["keys"][:nnz]), labels=blk["labels"][:used],
                     row_ptr=blk["row_ptr"][:used + 1], fgid=fgid, slice_rows=slice_rows)

    def _split(self, rows: int):
        """(used rows, slice rows) under the reference's slicing rule."""
        ts = rows // self.threads
        if self.cfg.keep_remainder:
            return rows, max(1, -(-rows // self.threads))
        return ts * self.threads, ts

    def _empty_batch(self) -> Batch:
        if getattr(self, "_empty", None) is None:
            self._empty = self._to_batch(None, 0, self.S)
        return self._empty

    def _epoch_batches(self, nxt, record):
        """This rank's batches of one epoch: blocks from ``nxt()`` (None at
        the end), each as one concurrent step or one step per slice."""
        while True:
            blk = nxt()
            if blk is None:
                return
            if self._resident is not None:
                batches = blk
            else:
                batches = list(self._slices_of(blk))
                if record is not None:
                    record.append(batches)
            yield from batches

    def _slices_of(self, blk: Optional[dict]):
        """Batches of one block: one concurrent step, or one step per slice."""
        rows = 0 if blk is None else (int(blk["rows"]) if "packed" in blk else len(blk["labels"]))
        if blk is not None and "packed" in blk and not self.concurrent:
            raise ValueError("packed .xfb shards train with concurrent slices (not --serial-slices)")
        used, sr = self._split(rows)
        if self.concurrent or blk is None or used <= 0:
            yield self._to_batch(blk, used, sr)
            return
        rp = np.asarray(blk.get("row_ptr_host", blk["row_ptr"]))
        for s0 in range(0, used, sr):
            n = min(sr, used - s0)
            k0, k1 = int(rp[s0]), int(rp[s0 + n])
            sub = {"row_ptr": blk["row_ptr"][s0: s0 + n + 1] - k0,
                   "keys": blk["keys"][k0: k1],
                   "fgid": blk["fgid"][k0: k1] if "fgid" in blk else None,
                   "labels": blk["labels"][s0: s0 + n]}
            if "row_ptr_host" in blk:
                sub["row_ptr_host"] = rp[s0: s0 + n + 1] - k0
                sub["nnz_per_row"] = blk["nnz_per_row"]
            yield self._to_batch(sub, n, n)

    # ----------------------------------------------------------------- train
    def init_push(self) -> None:
        """Reference initialisation pushes: key 0 (LR, FM: w and v) / key 1 (MVM)
        with zero gradients (lr_worker.cc:180-182, fm_worker.cc:248-252,
        mvm_worker.cc:276-278), applied once by the key's owner."""
        key = 1 if model_kind(self.cfg.model.kind) == 2 else 0
        if int(owner_of(np.array([key], dtype=np.uint64), self.world)[0]) == self.rank:
            self.table.push([key], np.zeros(self.table.params_per_key, dtype=np.float32))
        xdist.barrier()

    def train_epochs(self, epochs: int) -> None:
        cfg = self.cfg
        path = shard_path(cfg.train_prefix, self.rank)
        nat = _native.load()
        log_every = int(os.environ.get("XFLOW_LOG_EVERY", "0"))
        aps = self.aps
        for _ in range(epochs):
            if aps is not None:
                aps.resume()
            stream = record = None
            if self._resident is not None:  # batches kept in HBM by the first epoch
                blocks = iter(self._resident)
                nxt = lambda: next(blocks, None)  # noqa: E731
            else:
                xfb = binfmt.shard_file(path)
                # (on the CPU backend the same stream parses with reader.cpp's
                # rules through Engine.parse_text: the multi-rank gloo tests)
                gpu_text = cfg.gpu_parse and not xfb and self.concurrent
                reader = (binfmt.open_reader(xfb, self.block_rows) if xfb
                          else None if gpu_text
                          else nat.PrefetchReader(path, cfg.train_block_bytes))
                if gpu_text:
                    # libffm text tokenised on the GPU (data/textstream.py):
                    # the reference's blocks, parsed where they are trained
                    tl = (StreamTimeline(self.device)
                          if os.environ.get("XFLOW_STREAM_TIMELINE") else None)
                    stream = TextStream(self.engine, path, cfg.train_block_bytes,
                                        row_mod=1 if cfg.keep_remainder else self.threads,
                                        timeline=tl, read_threads=cfg.copy_threads)
                    nxt = stream.next
                else:
                    nxt = reader.next
                if reader is not None and self.device.type == "cuda" and self.concurrent:
                    # XFLOW_STREAM_TIMELINE=1: H2D vs step intervals from HIP
                    # events, reported in the epoch record (overlap evidence)
                    tl = (StreamTimeline(self.device)
                          if os.environ.get("XFLOW_STREAM_TIMELINE") else None)
                    stream = BlockStream(reader.next, self.device, self._with_fgid,
                                         copy_threads=cfg.copy_threads, timeline=tl)
                    nxt = stream.next
                record = [] if cfg.resident else None
            t0 = time.perf_counter()
            steps0 = self.steps
            ep_samples = 0
            sh = self.sharded
            w0 = ((sh.host_waits, sh.inline_prepares, sh.mid_step_waits, sh.host_wait_s)
                  if sh is not None else (0, 0, 0, 0.0))
            mw0 = self.engine.monitor_wait_seconds
            it = self._epoch_batches(nxt, record)
            empty = self._empty_batch()
            cur = next(it, None)
            while True:
                # multi-rank: the next batch is prepared inside this step and
                # the epoch ends when no rank has data (counts of -1)
                nb = next(it, None) if sh is not None else None
                if sh is None and cur is None:
                    break
                if self.watchdog is not None:
                    self.watchdog.beat()
                if cur is not None and not self.faults.before_step(self.steps) and sh is not None:
                    sh.drop_exchanges += 1  # fault injection: this rank skips an exchange
                tl = stream.timeline if stream is not None else None
                if tl is not None:
                    tl.begin("step")
                with self.timer.phase("step"):
                    if aps is not None:
                        if cur.rows > 0:
                            aps.train_step(cur)
                    elif sh is not None:
                        if not sh.train_step(cur if cur is not None else empty, S=self.S,
                                             next_batch=nb if nb is not None else empty):
                            break
                    elif cur.rows > 0:
                        self.engine.train_step(cur)
                if tl is not None:
                    tl.end("step")
                self.steps += 1
                ep_samples += cur.rows if cur is not None else 0
                if log_every and self.steps % log_every == 0:
                    self._log_progress(ep_samples, t0)
                cur = nb if sh is not None else next(it, None)
            timeline = None
            if stream is not None:
                stream.close()
                if stream.timeline is not None:
                    timeline = stream.timeline.overlap("h2d", "step")
                    timeline["host_stage_ms"] = 1000.0 * stream.stage_s
            if record is not None:
                self._resident = record
            if hasattr(self.sharded, "flush"):
                self.sharded.flush()
            if aps is not None:
                # every worker's pushes applied, every server idle: the table
                # shard is this thread's until the next epoch resumes serving
                aps.pause()
            self.samples += ep_samples
            self.epoch += 1
            if self.epoch % 30 == 0:
                _say("epoch : %d" % (self.epoch - 1))
            st = self.engine.read_stats(reset=True)
            tot = xdist.all_sum([st["ln_loss"], st["rows"], ep_samples,
                                 float(self.engine.overflowed() or self.table.overflowed())],
                                self.device)
            if tot[3] > 0:
                raise RuntimeError("table or dedup-scratch overflow during epoch %d: keys were "
                                   "dropped or isolated; grow --log2-cap / max_nnz" % self.epoch)
            keys = self.table.table_size()
            rec = dict(event="epoch", epoch=self.epoch, steps=self.steps,
                       train_logloss=tot[0] / max(tot[1], 1.0),
                       samples_per_s=tot[2] / max(time.perf_counter() - t0, 1e-9),
                       table_keys=keys, table_load=keys / float(self.table.table_capacity),
                       table_capacity=self.table.table_capacity,
                       table_growths=self.table.table_growths,
                       monitor_waits=self.table.monitor_waits)
            if aps is not None:
                rec["async_ps"] = {k: v for k, v in aps.stats().items()
                                   if k in ("max_staleness", "max_lead", "bytes_moved",
                                            "wait_pull_s", "wait_slot_s", "transport")}
            if timeline is not None:
                rec["timeline"] = {k: round(v, 3) for k, v in timeline.items()}
            # host time per step net of the time it sat blocked (monitor
            # run-ahead bound, split-size reads): what issuing a step costs
            ep_wall = time.perf_counter() - t0
            blocked = self.engine.monitor_wait_seconds - mw0 + (
                sh.host_wait_s - w0[3] if sh is not None else 0.0)
            n_ep = max(1, self.steps - steps0)
            rec["host_issue_ms_per_step"] = round(1000.0 * (ep_wall - blocked) / n_ep, 4)
            rec["host_blocked_ms_per_step"] = round(1000.0 * blocked / n_ep, 4)
            if sh is not None:
                # split-size reads that found the device copy in flight, and
                # steps whose batch was not prepared ahead (the epoch's first)
                rec["host_waits"] = sh.host_waits - w0[0]
                rec["inline_prepares"] = sh.inline_prepares - w0[1]
                # next-batch split-size reads inside a step that had to wait
                rec["mid_step_waits"] = sh.mid_step_waits - w0[2]
                rec["early_key_exchanges"] = getattr(sh, "early_key_exchanges", 0)
            if self.cfg.optim.lambda1 > 0 and os.environ.get("XFLOW_REPORT_NNZ"):
                rec["nonzero_weights"] = int(xdist.all_sum([self.table.nonzero_weights()],
                                                           self.device)[0])
            self.metrics.log(**rec)
            root = cfg.resume_dir or cfg.checkpoint_dir
            every = cfg.save_every or (1 if os.environ.get("XFLOW_CKPT_EVERY_EPOCH") else 0)
            if root and every and self.epoch % every == 0:
                self.save_versioned(root)
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)

    def _log_progress(self, ep_samples: int, t0: float) -> None:
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        rate = ep_samples / max(time.perf_counter() - t0, 1e-9)
        rec = dict(event="progress", epoch=self.epoch, step=self.steps, samples_per_s=rate,
                   unique_keys=self.engine.n_unique())
        if self.sharded is not None:
            rec["a2a_bytes"] = self.sharded.bytes_moved
        self.metrics.log(**rec)

    # --------------------------------------------------------------- predict
    def predict(self, block: int = 0) -> Optional[dict]:
        """Rank 0 predicts its test shard; other ranks serve their table shards.
        AUC / logloss are computed on the device (Engine.eval_metrics: radix
        sort + rank sums, csrc/hip/kernels_eval.hip); the predictions travel to
        the host only for the reference's pred_<rank>_<block>.txt file."""
        cfg = self.cfg
        nat = _native.load()
        dev_p, dev_y = [], []
        reader = None
        if self.rank == 0:
            tpath = shard_path(cfg.test_prefix, 0)
            xfb = binfmt.shard_file(tpath)
            reader = (binfmt.open_reader(xfb, self.block_rows) if xfb
                      else nat.BlockReader(tpath, cfg.resolved_test_block()))
        compat_mvm = model_kind(cfg.model.kind) == 2 and cfg.mvm_predict_compat
        aps = self.aps
        if aps is not None:
            aps.resume()  # every rank serves; rank 0's worker pulls over all of them
        while True:
            blk, used, sr = None, 0, 0
            while reader is not None:
                # (a block whose rows the slicing rule drops entirely -- fewer
                # rows than threads -- predicts nothing: skipped here, without
                # an exchange)
                blk = reader.next()
                if blk is None:
                    break
                used, sr = self._split(int(blk["rows"]) if "packed" in blk else len(blk["labels"]))
                if used > 0:
                    break
            if self.sharded is None and blk is None:
                break
            b = self._to_batch(blk, used, sr)
            if aps is not None:
                pctr = aps.eval_step(b) if b.rows > 0 else None
                if pctr is None:
                    continue
            elif self.sharded is not None:
                # every rank joins; "no test data left anywhere" travels in the
                # eval exchange's counts (no per-block collective)
                pctr = self.sharded.eval_step(b)
                if pctr is None:
                    break
            else:
                pctr = self.engine.eval_step(b)
            if b.rows == 0:
                continue
            p, y = pctr[:used], b.labels[:used]
            if compat_mvm and sr > 0:
                keep = torch.from_numpy((np.arange(used) % sr) < min(self.engine.model.v_dim, sr))
                keep = keep.to(p.device)
                p, y = p[keep], y[keep]
            dev_p.append(p.clone())
            dev_y.append(y.clone())
        if aps is not None:
            aps.pause()
        if self.rank != 0:
            return None
        dev = self.device
        p = torch.cat(dev_p) if dev_p else torch.zeros(0, dtype=torch.float32, device=dev)
        y = torch.cat(dev_y) if dev_y else torch.zeros(0, dtype=torch.float32, device=dev)
        res = self.engine.eval_metrics(p, y)
        dev_auc = res["auc"]
        if cfg.write_pred:
            os.makedirs(cfg.pred_dir or ".", exist_ok=True)
            ph, yh = p.cpu().numpy(), y.cpu().numpy().astype(np.int32)
            nat.write_pred(os.path.join(cfg.pred_dir or ".", "pred_%d_%d.txt" % (self.rank, block)),
                           np.ascontiguousarray(ph, dtype=np.float32), np.ascontiguousarray(yh))
            # predictions are on the host anyway: print the reference's exact
            # line, whose AUC depends on std::sort's (unspecified) order of
            # equal pctr values; the device AUC breaks ties by prediction order.
            # (Above 2^22 rows the host sort costs more than the whole device
            # eval and the reference's float accumulators drift: the device
            # line, exact sums, is printed instead.)
            if len(ph) <= (1 << 22):
                res = reference_auc(yh, ph)
        _say(res["line"])
        self.metrics.log(event="eval", auc=res["auc"], auc_device=dev_auc,
                         ln_logloss=res["ln_logloss"], logloss_printed=res["logloss_printed"],
                         n=res["n"])
        return res

    def train(self) -> Optional[dict]:
        """The reference's Worker::train(): log rank, train, rank-0 predict."""
        _say("my rank is = %d" % self.rank)
        if self.cfg.init_push and not self.resumed:
            self.init_push()
        # cfg.epochs counts the whole run: a resumed job trains the rest
        self.train_epochs(max(0, self.cfg.epochs - self.epoch) if self.resumed else self.cfg.epochs)
        res = None
        if self.rank == 0:
            _say("LR AUC: " if model_kind(self.cfg.model.kind) == 0 else "FM AUC: ")
        res = self.predict(0)
        _say("train end......")
        return res

    # ------------------------------------------------------------ checkpoint
    def save(self, ckpt_dir: str) -> None:
        if hasattr(self.sharded, "flush"):
            self.sharded.flush()
        checkpoint.save(self.table, ckpt_dir, self.rank, self.world,
                        meta={"epoch": self.epoch, "steps": self.steps}, barrier=xdist.barrier)
        xdist.barrier()

    def load(self, ckpt_dir: str) -> dict:
        meta = checkpoint.load(self.table, ckpt_dir, self.rank, self.world)
        self.epoch = int(meta.get("epoch", 0))
        self.steps = int(meta.get("steps", 0))
        xdist.barrier()
        return meta

    def save_versioned(self, root: str) -> None:
        """Periodic checkpoint: every rank writes its shard of this epoch's
        version, then rank 0 publishes it as LATEST (checkpoint.publish)."""
        self.save(checkpoint.version_dir(root, self.epoch))
        if self.rank == 0:
            checkpoint.publish(root, self.epoch)
        xdist.barrier()

    def resume(self, root: str) -> Optional[dict]:
        """Continue from root's newest complete versioned checkpoint, if any
        (the tracker's recovery path); later periodic saves go to root."""
        self.cfg.resume_dir = root
        d = checkpoint.latest(root)
        if d is None:
            return None
        meta = self.load(d)
        self.resumed = True
        _say("resumed from %s at epoch %d" % (d, self.epoch))
        return meta

    def close(self) -> None:
        if self.watchdog is not None:
            self.watchdog.stop()
        if getattr(self, "sharded", None) is not None:
            self.sharded.close()
        if getattr(self, "aps", None) is not None:
            self.aps.close()
        xdist.finalize()


if __name__ == "__main__":  # pragma: no cover
    sys.exit("use python -m xflow_amd.cli")
