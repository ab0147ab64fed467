"""Plain-PyTorch fp32 reference of one training step (numerics oracle for the
HIP / C++ engine).  Independent implementation: torch.unique for dedup,
index_add for the per-row sums and per-(key, slice) gradient sums, vectorised
FTRL-Proximal / SGD closed forms.  Semantics: all slices of a batch read the
same weights; gradients are per-slice sums divided by slice rows
(lr_worker.cc:100-119); each slice's push is applied in slice order
(ftrl.h:58-74).  Covers LR / FM (reference + standard math) / MVM.
"""
from __future__ import annotations

import math

import numpy as np
import torch

LN_BASE = math.log(2.718281828)


def sigmoid_ref(x: torch.Tensor) -> torch.Tensor:
    xd = x.double()
    ex = torch.exp(xd * LN_BASE)
    p = (ex / (1.0 + ex)).float()
    p = torch.where(x < -30, torch.full_like(p, 1e-6), p)
    p = torch.where(x > 30, torch.ones_like(p), p)
    return p


class RefTable:
    """Sorted-key table of FTRL (n, z) or SGD w state, P params per key."""

    def __init__(self, P: int, p_w: int, opt: str = "ftrl", alpha=5e-2, beta=1.0, l1=5e-5,
                 l2=10.0, lr=1e-3, sgd_v_init=1e-3, init_fn=None):
        self.P, self.p_w, self.opt = P, p_w, opt
        self.alpha, self.beta, self.l1, self.l2, self.lr = alpha, beta, l1, l2, lr
        self.sgd_v_init = sgd_v_init
        self.init_fn = init_fn          # (keys np.uint64, dim) -> float32 init of latent params
        self.keys = np.zeros(0, dtype=np.uint64)
        sw = 2 if opt == "ftrl" else 1
        self.state = torch.zeros((0, P * sw), dtype=torch.float32)
        self.pushed = torch.zeros(0, dtype=torch.bool)

    def _rows(self, keys: np.ndarray, insert: bool) -> np.ndarray:
        idx = np.searchsorted(self.keys, keys)
        found = (idx < len(self.keys)) & (self.keys[np.minimum(idx, len(self.keys) - 1)] == keys) \
            if len(self.keys) else np.zeros(len(keys), dtype=bool)
        if insert and not found.all():
            new = np.unique(keys[~found])
            allk = np.concatenate([self.keys, new])
            order = np.argsort(allk, kind="stable")
            self.keys = allk[order]
            st = torch.cat([self.state, torch.zeros((len(new), self.state.shape[1]))])
            pu = torch.cat([self.pushed, torch.zeros(len(new), dtype=torch.bool)])
            o = torch.from_numpy(order)
            self.state, self.pushed = st[o], pu[o]
            return self._rows(keys, False)
        idx = idx.copy()
        idx[~found] = -1
        return idx

    def _latent_init(self, keys: np.ndarray, p: int) -> torch.Tensor:
        if self.opt == "sgd":
            return torch.full((len(keys),), self.sgd_v_init)
        return torch.from_numpy(self.init_fn(keys, p - self.p_w)).float()

    def weights(self, keys: np.ndarray, insert: bool = True) -> torch.Tensor:
        rows = self._rows(keys, insert)
        out = torch.zeros((len(keys), self.P))
        present = torch.from_numpy(rows >= 0)
        r = torch.from_numpy(np.maximum(rows, 0))
        for p in range(self.P):
            if self.opt == "ftrl":
                n, z = self.state[r, 2 * p], self.state[r, 2 * p + 1]
                w = self._ftrl_w(z, n)
            else:
                w = self.state[r, p]
            if p >= self.p_w:
                init = self._latent_init(keys, p)
                use_init = ~present | ~self.pushed[r]
                w = torch.where(use_init, init, w)
            elif not bool(present.all()):
                w = torch.where(present, w, torch.zeros_like(w))
            out[:, p] = w
        return out

    def _ftrl_w(self, z, n):
        a = torch.tensor(self.alpha, dtype=torch.float32)
        tmpr = torch.where(z > 0, z - self.l1, torch.where(z < 0, z + self.l1, torch.zeros_like(z)))
        tmpl = -1.0 * ((self.beta + torch.sqrt(n)) / a + self.l2)
        return torch.where(z.abs() <= self.l1, torch.zeros_like(z), tmpr / tmpl)

    def push(self, keys: np.ndarray, g: torch.Tensor) -> None:
        """One push per key (keys unique), g: [len(keys), P]."""
        rows = torch.from_numpy(self._rows(keys, True))
        w = self.weights(keys, insert=False)
        for p in range(self.P):
            if self.opt == "ftrl":
                n = self.state[rows, 2 * p]
                z = self.state[rows, 2 * p + 1]
                gp = g[:, p]
                nn = n + gp * gp
                z = z + (gp - (torch.sqrt(nn) - torch.sqrt(n)) / self.alpha * w[:, p])
                self.state[rows, 2 * p] = nn
                self.state[rows, 2 * p + 1] = z
            else:
                self.state[rows, p] = w[:, p] - self.lr * g[:, p]
        self.pushed[rows] = True


def forward(kind: str, W: torch.Tensor, inv: torch.Tensor, row_of: torch.Tensor, rows: int,
            fgid: torch.Tensor | None = None, fm_math: str = "reference", mvm_math: str = "compat"):
    """Returns (y logits [rows], aux) with W = pulled params per unique key."""
    if kind == "lr":
        y = torch.zeros(rows).index_add_(0, row_of, W[inv, 0])
        return y, None
    if kind == "fm":
        D = W.shape[1] - 1
        wx = torch.zeros(rows).index_add_(0, row_of, W[inv, 0])
        V = W[inv, 1:]
        vs = torch.zeros((rows, D)).index_add_(0, row_of, V)
        vp = torch.zeros(rows).index_add_(0, row_of, (V * V).sum(1))
        if fm_math == "standard":
            y = wx + 0.5 * ((vs * vs).sum(1) - vp)
        else:
            tot = vs.sum(1)
            y = wx + (tot * tot - vp)
        return y, vs
    # mvm
    D = W.shape[1]
    G = int(fgid.max().item()) + 2 if fgid.numel() else 1
    S = torch.zeros((rows, G, D))
    flat = row_of * G + fgid.long()
    S.view(rows * G, D).index_add_(0, flat, W[inv])
    maxf = torch.zeros(rows, dtype=torch.long).scatter_reduce_(0, row_of, fgid.long(), "amax")
    gidx = torch.arange(G).unsqueeze(0)
    lim = maxf if mvm_math == "compat" else maxf + 1
    mask = (gidx < lim.unsqueeze(1)).unsqueeze(2)
    M = torch.where(mask, S, torch.ones_like(S)).prod(1)
    return M.sum(1), (S, M)


def train_step(table: RefTable, kind: str, keys: np.ndarray, labels: np.ndarray,
               row_ptr: np.ndarray, slice_rows: int, fgid: np.ndarray | None = None,
               fm_math: str = "reference", mvm_math: str = "compat", sum_slices: bool = False):
    """One engine-semantics step; returns pctr [rows]."""
    p, pending = compute_step(table, kind, keys, labels, row_ptr, slice_rows, fgid, fm_math,
                              mvm_math)
    apply_step(table, pending, sum_slices)
    return p


def apply_step(table: RefTable, pending, sum_slices: bool = False) -> None:
    """Push a compute_step's per-(key, slice) gradients in slice order."""
    uniq, g, touched = pending
    nS = g.shape[1]
    if sum_slices:
        gg = torch.where(touched.unsqueeze(2), g, torch.zeros_like(g)).sum(1)
        table.push(uniq, gg)
        return
    for s in range(nS):
        sel = touched[:, s].numpy()
        if sel.any():
            table.push(uniq[sel], g[torch.from_numpy(sel), s])


def compute_step(table: RefTable, kind: str, keys: np.ndarray, labels: np.ndarray,
                 row_ptr: np.ndarray, slice_rows: int, fgid: np.ndarray | None = None,
                 fm_math: str = "reference", mvm_math: str = "compat"):
    """Pull + forward + backward of one step; returns (pctr, pending pushes)."""
    rows = len(labels)
    counts = np.diff(row_ptr)
    row_of = torch.from_numpy(np.repeat(np.arange(rows), counts)).long()
    uniq, inv = np.unique(keys, return_inverse=True)
    inv = torch.from_numpy(inv.reshape(-1)).long()
    W = table.weights(uniq, insert=True)
    fg = torch.from_numpy(fgid).long() if fgid is not None else None
    y, aux = forward(kind, W, inv, row_of, rows, fg, fm_math, mvm_math)
    p = sigmoid_ref(y)
    loss = p - torch.from_numpy(labels).float()
    lo = loss[row_of]
    P = table.P
    if kind == "lr":
        contrib = lo.unsqueeze(1)
    elif kind == "fm":
        D = P - 1
        V = W[inv, 1:]
        if fm_math == "standard":
            ref = aux[row_of]
            gw = lo
        else:
            ref = aux.sum(1)[row_of].unsqueeze(1)
            gw = lo * float(D)
        contrib = torch.cat([gw.unsqueeze(1), lo.unsqueeze(1) * (ref - V)], 1)
    else:
        S, M = aux
        G = S.shape[1]
        sg = S.view(rows * G, -1)[row_of * G + fg]
        Mo = M[row_of]
        gr = (lo.double().unsqueeze(1) * (Mo.double() / (1.0 + sg.double()))).float()
        contrib = torch.where(sg == 0, torch.zeros_like(gr), gr)
    nS = (rows + slice_rows - 1) // slice_rows if slice_rows > 0 else 1
    sl = (row_of // slice_rows).clamp(max=nS - 1) if slice_rows > 0 else torch.zeros_like(row_of)
    U = len(uniq)
    gsum = torch.zeros((U * nS, P)).index_add_(0, inv * nS + sl, contrib).view(U, nS, P)
    touched = torch.zeros(U * nS).index_add_(0, inv * nS + sl, torch.ones(len(inv))).view(U, nS) > 0
    srows = [min(slice_rows, rows - s * slice_rows) if slice_rows > 0 else rows for s in range(nS)]
    norm = torch.tensor(srows, dtype=torch.float64)
    g = (gsum.double() / norm.view(1, nS, 1)).float()
    return p, (uniq, g, touched)
