"""BlockInfo, get_block_info and the greedy weight balancer (MPMP.jl:425-560), 0-based.

The balancer is reused for the cluster -> GPU map: the reference balances
(j,l) pairs over threads by ``Y_blocksize^3`` (MPMP.jl:495-499); :func:`partition_clusters`
balances whole clusters over ranks with the per-cluster cost of one iteration.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import List, Sequence


def distribute_weights_swapping(weights, n, nswaps=None):
    """Greedy swap balance of ``weights`` over ``n`` sets (MPMP.jl:425-465).

    Starts from contiguous sets of size ``len//n + 1`` and ``len//n`` and swaps the heaviest
    element of the heaviest set with the lightest element of the lightest set while that lowers
    the maximum.  Returns ``(sets, set_weights)`` with 0-based element indices.
    """
    w = list(weights)
    if nswaps is None:
        nswaps = len(w) ** 2
    step = len(w) // n + 1
    nstep = n - (step * n - len(w))
    sets = [list(range(i * step, (i + 1) * step)) for i in range(nstep)]
    sets += [list(range(nstep * step + i * (step - 1), nstep * step + (i + 1) * (step - 1)))
             for i in range(n - nstep)]
    set_w = [sum(w[i] for i in s) for s in sets]
    index_set, index_el = 1, 1
    for _ in range(nswaps):
        order = sorted(((set_w[i], i) for i in range(len(set_w))), reverse=True)
        max_set = order[index_set - 1][1]
        if not sets[max_set]:
            break
        els = sorted(((w[sets[max_set][i]], i) for i in range(len(sets[max_set]))), reverse=True)
        if index_el - 1 >= len(els):
            break
        max_el = sets[max_set][els[index_el - 1][1]]
        min_set = min(range(len(set_w)), key=lambda i: set_w[i])
        if not sets[min_set]:
            # an empty set (more sets than weights): move instead of swap
            if set_w[max_set] - w[max_el] < set_w[max_set] and len(sets[max_set]) > 1:
                sets[max_set].remove(max_el)
                sets[min_set].append(max_el)
                set_w[max_set] -= w[max_el]
                set_w[min_set] += w[max_el]
                continue
            break
        min_el = min(sets[min_set], key=lambda i: w[i])
        if (set_w[min_set] + w[max_el] - w[min_el] < set_w[max_set]
                and set_w[max_set] - w[max_el] + w[min_el] < set_w[max_set]):
            sets[max_set] = [i for i in sets[max_set] if i != max_el] + [min_el]
            set_w[max_set] += w[min_el] - w[max_el]
            sets[min_set] = [i for i in sets[min_set] if i != min_el] + [max_el]
            set_w[min_set] += w[max_el] - w[min_el]
            index_el, index_set = 1, 1
        elif index_el < len(sets[index_set - 1]):
            index_el += 1
        elif index_el == step - 1 and index_set < n - 1:
            index_set += 1
            index_el = 1
        else:
            break
    return sets, set_w


@dataclass
class BlockInfo:
    """Sizes and ranks of a clustered low-rank SDP (MPMP.jl:467-513), 0-based indices."""

    J: int
    n_y: int
    m: List[int]
    L: List[int]
    n_samples: List[int]
    Y_blocksizes: List[List[int]]
    dim_S: List[int]
    ranks: List[List[List[int]]]
    x_indices: List[int] = field(default_factory=list)
    rank_sums: list = field(default_factory=list)
    nz_k: list = field(default_factory=list)
    jl_pairs: list = field(default_factory=list)

    def __post_init__(self):
        J = self.J
        if not (len(self.m) == len(self.L) == len(self.n_samples) == len(self.dim_S) == J):
            raise ValueError("sizes of m,L,n_samples,dim_S must equal the number of constraints")
        if [len(r) for r in self.ranks] != list(self.L) or \
                [len(y) for y in self.Y_blocksizes] != list(self.L):
            raise ValueError("Y[j] and ranks[j] must have length L[j]")
        self.x_indices = [sum(self.dim_S[:j]) for j in range(J + 1)]
        self.rank_sums = [[[0] + _cumsum(self.ranks[j][l]) for l in range(self.L[j])]
                          for j in range(J)]
        self.nz_k = [[next(k for k in range(self.n_samples[j]) if self.ranks[j][l][k] > 0)
                      for l in range(self.L[j])] for j in range(J)]
        self.jl_pairs = [(j, l) for j in range(J) for l in range(self.L[j])]

    @property
    def total_dim(self) -> int:
        """size(X, 1) (MPMP.jl:716)."""
        return sum(sum(b) for b in self.Y_blocksizes)


def _cumsum(v):
    out, s = [], 0
    for x in v:
        s += x
        out.append(s)
    return out


def block_info(J, n_y, m, L, n_samples, Y_blocksizes, ranks) -> BlockInfo:
    """BlockInfo(J, n_y, m, L, n_samples, Y_blocksizes, ranks) (MPMP.jl:504-513)."""
    dim_S = [m[j] * (m[j] + 1) // 2 * n_samples[j] for j in range(J)]
    return BlockInfo(J, n_y, list(m), list(L), list(n_samples), Y_blocksizes, dim_S, ranks)


def get_block_info(constraints: Sequence) -> BlockInfo:
    """Extract BlockInfo from the (A, B, c, H) constraint tuples (MPMP.jl:516-560)."""
    J = len(constraints)
    n_y = constraints[0][1].shape[1]
    L = [len(constraints[j][0]) for j in range(J)]
    n_samples = [len(constraints[j][0][0]) for j in range(J)]
    m = [(-1 + math.isqrt(8 * (len(constraints[j][2]) // n_samples[j]) + 1)) // 2
         for j in range(J)]
    for j in range(J):
        if len(constraints[j][2]) != m[j] * (m[j] + 1) * n_samples[j] // 2:
            raise ValueError(f"cluster {j}: len(c) is not m(m+1)/2 * n_samples")
    ranks = [[[len(constraints[j][0][l][k]) for k in range(n_samples[j])] for l in range(L[j])]
             for j in range(J)]
    nz = [[next(k for k in range(n_samples[j]) if ranks[j][l][k] > 0) for l in range(L[j])]
          for j in range(J)]
    Yb = [[m[j] * len(constraints[j][0][l][nz[j][l]][0]) for l in range(L[j])] for j in range(J)]
    return block_info(J, n_y, m, L, n_samples, Yb, ranks)


def cluster_cost(bi: BlockInfo, j: int) -> float:
    """Model flops of one iteration spent on cluster j (Schur pairings + chol(S_j) + L^-1 B_j +
    the cubic block work), the weight of the cluster -> rank balancer."""
    D = bi.dim_S[j]
    c = D ** 3 / 3.0 + 2.0 * D * D * bi.n_y
    for l in range(bi.L[j]):
        n = bi.Y_blocksizes[j][l]
        m = bi.m[j]
        K = bi.rank_sums[j][l][-1]
        delta = n // m
        c += 4.0 * m * m * delta * K * (delta + K) + 30.0 * n ** 3
    return c


def partition_clusters(bi: BlockInfo, world: int) -> List[List[int]]:
    """Clusters -> ranks with the reference's balancer (MPMP.jl:425-465) on cluster_cost."""
    if world <= 1:
        return [list(range(bi.J))]
    w = [cluster_cost(bi, j) for j in range(bi.J)]
    sets, _ = distribute_weights_swapping(w, world, nswaps=len(w) ** 2)
    return [sorted(s) for s in sets]
