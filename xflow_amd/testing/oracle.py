"""Pure-Python oracle of the reference's behaviour,
written from the reference sources, independent of the engine:

* reader: libffm lines, label atof > 1e-7, fid = std::hash of the fid text
  (load_data_from_disk.cc:103-210);
* slicing: rows // threads rows per slice, remainder dropped (lr_worker.cc:190);
* per slice: sorted unique keys, Pull, loss, per-key gradient sums / rows,
  Push (lr_worker.cc:145-177; fm_worker.cc:204-245; mvm_worker.cc:220-273);
* FTRL-Proximal handle (ftrl.h:38-152) and SGD handle (sgd.h:30-109) on a
  dict store, float32 arithmetic;
* predict + calculate_auc (base.h:84-110).

Slices are executed serially (slice i+1 pulls after slice i pushed), the
deterministic schedule of the reference's Hogwild threads; with
``concurrent=True`` all slices of a block pull first, then push in order.
Latent (v) parameters take their initial value from ``v_init(key, k)``.
"""
from __future__ import annotations

import math
from typing import Callable, Dict, List, Optional, Tuple

import numpy as np

from xflow_amd.testing.hashing import std_hash

F32 = np.float32


def parse_file(path: str) -> List[Tuple[int, List[Tuple[int, int]]]]:
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


def sigmoid(x: float) -> float:
    x = float(F32(x))
    if x < -30:
        return float(F32(1e-6))
    if x > 30:
        return 1.0
    ex = math.pow(2.718281828, x)
    return float(F32(ex / (1.0 + ex)))


class Store:
    """ps-lite KVServer store with the FTRL or SGD request handle."""

    def __init__(self, P: int, p_w: int, opt: str = "ftrl",
                 v_init: Optional[Callable[[int, int], float]] = None,
                 alpha=5e-2, beta=1.0, l1=5e-5, l2=10.0, lr=1e-3, sgd_v=1e-3):
        self.P, self.p_w, self.opt = P, p_w, opt
        self.v_init = v_init or (lambda key, k: 0.0)
        self.a, self.b, self.l1, self.l2, self.lr, self.sgd_v = \
            F32(alpha), F32(beta), F32(l1), F32(l2), F32(lr), F32(sgd_v)
        self.w: Dict[int, np.ndarray] = {}
        self.n: Dict[int, np.ndarray] = {}
        self.z: Dict[int, np.ndarray] = {}

    def _entry(self, key: int):
        if key not in self.w:
            w = np.zeros(self.P, dtype=F32)
            for p in range(self.p_w, self.P):
                w[p] = F32(self.v_init(key, p - self.p_w)) if self.opt == "ftrl" else self.sgd_v
            self.w[key] = w
            self.n[key] = np.zeros(self.P, dtype=F32)
            self.z[key] = np.zeros(self.P, dtype=F32)
        return self.w[key], self.n[key], self.z[key]

    def pull(self, keys) -> np.ndarray:
        return np.stack([self._entry(k)[0].copy() for k in keys]) if keys else \
            np.zeros((0, self.P), F32)

    def push(self, keys, grads: np.ndarray) -> None:
        for i, k in enumerate(keys):
            w, n, z = self._entry(k)
            for j in range(self.P):
                g = F32(grads[i, j])
                if self.opt == "sgd":
                    w[j] = F32(w[j] - self.lr * g)
                    continue
                old_n = n[j]
                nn = F32(old_n + g * g)
                z[j] = F32(z[j] + F32(g - F32(F32(np.sqrt(nn) - np.sqrt(old_n)) / self.a) * w[j]))
                n[j] = nn
                if abs(z[j]) <= self.l1:
                    w[j] = F32(0.0)
                else:
                    tmpr = F32(z[j] - self.l1) if z[j] > 0 else F32(z[j] + self.l1)
                    tmpl = F32(-1.0) * F32(F32(self.b + np.sqrt(n[j])) / self.a + self.l2)
                    w[j] = F32(tmpr / tmpl)


def _forward(kind: str, rows, W: Dict[int, np.ndarray], D: int, fm_math: str, mvm_math: str):
    """Per-row logits and the auxiliaries the gradients need."""
    out, aux = [], []
    for _, feats in rows:
        if kind == "lr":
            y = F32(0)
            for _, k in feats:
                y = F32(y + W[k][0])
            out.append(y)
            aux.append(None)
        elif kind == "fm":
            wx, vp = F32(0), F32(0)
            vs = np.zeros(D, F32)
            for _, k in feats:
                wx = F32(wx + W[k][0])
                for d in range(D):
                    v = W[k][1 + d]
                    vs[d] = F32(vs[d] + v)
                    vp = F32(vp + v * v)
            if fm_math == "standard":
                y = F32(wx + F32(0.5) * F32(F32((vs * vs).sum()) - vp))
                aux.append(vs)
            else:
                tot = F32(vs.sum())
                y = F32(wx + F32(tot * tot - vp))
                aux.append(tot)
            out.append(y)
        else:
            maxf = max((g for g, _ in feats), default=0)
            G = maxf if mvm_math == "compat" else maxf + 1
            S = np.zeros((maxf + 1, D), F32)
            for g, k in feats:
                S[g] = S[g] + W[k]
            M = np.ones(D, F32)
            for g in range(G):
                M = (M * S[g]).astype(F32)
            y = F32(0)
            for d in range(D):
                y = F32(y + M[d])
            out.append(y)
            aux.append((S, M))
    return out, aux


def _grads(kind, rows, W, loss, aux, D, fm_math) -> Dict[int, np.ndarray]:
    P = len(next(iter(W.values()))) if W else 1
    g: Dict[int, np.ndarray] = {}
    for (_, feats), lo, ax in zip(rows, loss, aux):
        for fg, k in feats:
            acc = g.setdefault(k, np.zeros(P, np.float64))
            if kind == "lr":
                acc[0] += lo
            elif kind == "fm":
                acc[0] += lo * (1 if fm_math == "standard" else D)
                for d in range(D):
                    ref = ax[d] if fm_math == "standard" else ax
                    acc[1 + d] += lo * (ref - W[k][1 + d])
            else:
                S, M = ax
                for d in range(D):
                    sg = S[fg][d]
                    acc[d] += 0.0 if sg == 0 else float(F32(lo * (M[d] / (1.0 + sg))))
    return g


class Oracle:
    def __init__(self, kind: str = "lr", opt: str = "ftrl", v_dim: int = 10,
                 fm_math: str = "reference", mvm_math: str = "compat", threads: int = 8,
                 v_init=None, concurrent: bool = False):
        self.kind, self.D, self.fm_math, self.mvm_math = kind, v_dim, fm_math, mvm_math
        self.threads, self.concurrent = threads, concurrent
        P = 1 if kind == "lr" else (1 + v_dim if kind == "fm" else v_dim)
        self.store = Store(P, 0 if kind == "mvm" else 1, opt, v_init)

    def init_push(self) -> None:
        key = 1 if self.kind == "mvm" else 0
        self.store.push([key], np.zeros((1, self.store.P), F32))

    def _slice_step(self, rows, W=None) -> None:
        keys = sorted({k for _, f in rows for _, k in f})
        if W is None:
            W = dict(zip(keys, self.store.pull(keys)))
        logits, aux = _forward(self.kind, rows, W, self.D, self.fm_math, self.mvm_math)
        loss = [float(F32(sigmoid(y) - lab)) for y, (lab, _) in zip(logits, rows)]
        g = _grads(self.kind, rows, W, loss, aux, self.D, self.fm_math)
        n = len(rows)
        grads = np.stack([(g[k] / n).astype(F32) for k in keys]) if keys else None
        if keys:
            self.store.push(keys, grads)

    def train_block(self, rows) -> None:
        ts = len(rows) // self.threads
        if ts == 0:
            return
        slices = [rows[i * ts:(i + 1) * ts] for i in range(self.threads)]
        if not self.concurrent:
            for s in slices:
                self._slice_step(s)
            return
        keys = sorted({k for _, f in rows[: ts * self.threads] for _, k in f})
        W = dict(zip(keys, self.store.pull(keys)))
        for s in slices:
            self._slice_step(s, {k: W[k] for _, f in s for _, k in f})

    def predict(self, rows) -> List[Tuple[int, float]]:
        ts = len(rows) // self.threads
        used = rows[: ts * self.threads]
        keys = sorted({k for _, f in used for _, k in f})
        W = dict(zip(keys, self.store.pull(keys)))
        logits, _ = _forward(self.kind, used, W, self.D, self.fm_math, self.mvm_math)
        return [(lab, sigmoid(y)) for y, (lab, _) in zip(logits, used)]


def calculate_auc(pairs: List[Tuple[int, float]]) -> Tuple[float, float]:
    """(printed signed mean log2-likelihood, auc) as base.h:84-110."""
    v = sorted(pairs, key=lambda t: -t[1])
    area, tp, ll = 0.0, 0, F32(0)
    for lab, p in v:
        if lab == 1:
            tp += 1
        else:
            area += tp
        with np.errstate(divide="ignore"):
            ll = F32(ll + lab * math.log2(p) + (1.0 - lab) * math.log2(1.0 - p)
                     if p not in (0.0, 1.0) else ll)
    ll = F32(ll / len(v))
    auc = area / (tp * (len(v) - tp)) if 0 < tp < len(v) else float("nan")
    return float(ll), auc
