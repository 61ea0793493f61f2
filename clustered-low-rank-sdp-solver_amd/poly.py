"""Sparse multivariate polynomials with mpmath coefficients, and the reference's bases and
sample points (MPMP.jl:21-200).

The reference builds its constraint data with AbstractAlgebra.jl polynomials (``PolynomialRing``
over ``RealField``) and evaluates them at BigFloat sample points.  ``prepareabc`` only needs
evaluation at a point, ``total_degree``, ``coeffs`` and ring arithmetic to build the inputs, so
:class:`Poly` is a dictionary ``{exponent tuple: mpf}`` with exactly those operations.  All
arithmetic runs at the current ``mpmath.mp.prec`` (the reference's ``precision(BigFloat)``).
"""
from __future__ import annotations

import itertools
import math
from typing import Dict, Iterable, List, Sequence, Tuple

import mpmath
from mpmath import mp, mpf


class Poly:
    """A polynomial in ``nvars`` variables: ``terms[exponent] = coefficient``."""

    __slots__ = ("nvars", "terms")

    def __init__(self, nvars: int = 1, terms: Dict[Tuple[int, ...], object] | None = None):
        self.nvars = nvars
        self.terms = {}
        for e, c in (terms or {}).items():
            c = mpf(c)
            if c != 0:
                self.terms[tuple(e)] = c

    # -- constructors
    @classmethod
    def const(cls, c, nvars: int = 1) -> "Poly":
        return cls(nvars, {(0,) * nvars: c})

    @classmethod
    def gens(cls, nvars: int) -> List["Poly"]:
        """The ring generators x_1..x_n (AbstractAlgebra ``gens``)."""
        return [cls(nvars, {tuple(1 if i == j else 0 for i in range(nvars)): 1})
                for j in range(nvars)]

    @classmethod
    def monomial(cls, exponent: Sequence[int], c=1) -> "Poly":
        return cls(len(exponent), {tuple(exponent): c})

    # -- queries
    def total_degree(self) -> int:
        """AbstractAlgebra ``total_degree``: -1 for the zero polynomial."""
        return max((sum(e) for e in self.terms), default=-1)

    def coeffs(self) -> List[object]:
        return list(self.terms.values())

    def is_zero(self) -> bool:
        return not self.terms

    def __call__(self, *x):
        """Evaluate at a point (scalars or one sequence); ``q(x[k]...)`` in the reference."""
        if len(x) == 1 and isinstance(x[0], (list, tuple)):
            x = tuple(x[0])
        if len(x) != self.nvars:
            raise ValueError(f"polynomial in {self.nvars} variables evaluated at {len(x)} values")
        xs = [mpf(v) for v in x]
        s = mpf(0)
        for e, c in self.terms.items():
            t = c
            for xi, ei in zip(xs, e):
                if ei:
                    t *= xi ** ei
            s += t
        return s

    # -- arithmetic
    def _lift(self, o) -> "Poly":
        return o if isinstance(o, Poly) else Poly.const(o, self.nvars)

    def __add__(self, o):
        o = self._lift(o)
        t = dict(self.terms)
        for e, c in o.terms.items():
            t[e] = t.get(e, mpf(0)) + c
        return Poly(self.nvars, t)

    __radd__ = __add__

    def __neg__(self):
        return Poly(self.nvars, {e: -c for e, c in self.terms.items()})

    def __sub__(self, o):
        return self + (-self._lift(o))

    def __rsub__(self, o):
        return self._lift(o) - self

    def __mul__(self, o):
        if not isinstance(o, Poly):
            o = mpf(o)
            return Poly(self.nvars, {e: c * o for e, c in self.terms.items()})
        t: Dict[Tuple[int, ...], object] = {}
        for e1, c1 in self.terms.items():
            for e2, c2 in o.terms.items():
                e = tuple(a + b for a, b in zip(e1, e2))
                t[e] = t.get(e, mpf(0)) + c1 * c2
        return Poly(self.nvars, t)

    __rmul__ = __mul__

    def __truediv__(self, o):
        return self * (mpf(1) / mpf(o))

    def __pow__(self, k: int):
        r = Poly.const(1, self.nvars)
        for _ in range(int(k)):
            r = r * self
        return r

    def __repr__(self):
        if not self.terms:
            return "0"
        return " + ".join(f"{mpmath.nstr(c, 8)}*x^{e}" for e, c in sorted(self.terms.items()))


def evaluate(p, point):
    """``p(point...)`` for a Poly or a plain number (constant entries of the reference's
    matrices, e.g. ``S1(constant)``)."""
    if isinstance(p, Poly):
        return p(point)
    return mpf(p)


def total_degree(p) -> int:
    if isinstance(p, Poly):
        return p.total_degree()
    return -1 if mpf(p) == 0 else 0


# ---------------------------------------------------------------------------------------------
# bases (MPMP.jl:21-89)
# ---------------------------------------------------------------------------------------------
def multiexponents(n: int, k: int) -> Iterable[Tuple[int, ...]]:
    """Exponent vectors of length n and total degree k in Combinatorics.jl's order
    (reverse-lexicographic: (k,0,..,0) first)."""
    if n == 1:
        yield (k,)
        return
    for first in range(k, -1, -1):
        for rest in multiexponents(n - 1, k - first):
            yield (first,) + rest


def make_monomial_basis(nvars: int, d: int) -> List[Poly]:
    """Monomial basis up to total degree d (MPMP.jl:23-40), ``binomial(n+d, d)`` polynomials."""
    q = []
    for k in range(d + 1):
        for e in multiexponents(nvars, k):
            q.append(Poly.monomial(e))
    assert len(q) == math.comb(nvars + d, d)
    return q


def laguerrebasis(k: int, alpha, x):
    """Laguerre polynomials L_0..L_k^{alpha}(x) by the three-term recurrence (MPMP.jl:42-53).
    ``x`` may be a number or a :class:`Poly`."""
    one = Poly.const(1, x.nvars) if isinstance(x, Poly) else mpf(1)
    alpha = mpf(alpha)
    v = [one]
    if k == 0:
        return v
    v.append(1 + alpha - x)
    for l in range(2, k + 1):
        v.append(((2 * l - 1 + alpha - x) * v[l - 1] - (l + alpha - 1) * v[l - 2]) * (mpf(1) / l))
    return v


def jacobi_basis(d: int, alpha, beta, x, normalized: bool = True):
    """MPMP.jl:55-74, restated with the recurrence exactly as written there."""
    one = Poly.const(1, x.nvars) if isinstance(x, Poly) else mpf(1)
    alpha, beta = mpf(alpha), mpf(beta)
    q = [one]
    if d == 0:
        return q
    q.append(x if normalized else x * (alpha + 1))
    for k in range(2, d + 1):
        c = (2 * k + alpha + beta - 1) / (mpf(2 * k) * (k + alpha + beta) * (2 * k + alpha + beta - 2))
        q.append(c * ((2 * k + alpha + beta) * (2 * k + alpha + beta - 2) * x + beta ** 2 - alpha ** 2)
                 * q[k - 1] + (-2 * (k + alpha - 1) * (k + beta - 1) * (2 * k + alpha + beta)) * q[k - 2])
    return q


def gegenbauer_basis(k: int, n: int, x):
    """Gegenbauer polynomials for dimension n, normalised to 1 at 1 (MPMP.jl:76-89)."""
    one = Poly.const(1, x.nvars) if isinstance(x, Poly) else mpf(1)
    v = [one]
    if k == 0:
        return v
    v.append(x)
    for l in range(2, k + 1):
        v.append(mpf(2 * l + n - 4) / (l + n - 3) * x * v[l - 1] - mpf(l - 1) / (l + n - 3) * v[l - 2])
    return v


# ---------------------------------------------------------------------------------------------
# sample points (MPMP.jl:91-200)
# ---------------------------------------------------------------------------------------------
def create_sample_points(n: int, d: int) -> List[List[object]]:
    """Rational points of the unit simplex with denominator d (MPMP.jl:91-103), in Julia's
    CartesianIndices order (first coordinate fastest)."""
    out = []
    for idx in itertools.product(range(d + 1), repeat=n):
        I = idx[::-1]
        if sum(I) <= d:
            out.append([mpf(i) / d for i in I])
    assert len(out) == math.comb(n + d, d)
    return out


def create_sample_points_2d(d: int) -> List[List[object]]:
    """Padua points (MPMP.jl:105-120)."""
    z = []
    for j in range(d + 1):
        delta_j = 1 if (j % 2 == 1 and d % 2 == 1) else 0
        mu_j = mpmath.cospi(mpf(j) / d)
        for k in range(1, d // 2 + 1 + delta_j + 1):
            if j % 2 == 1:
                eta = mpmath.cospi(mpf(2 * k - 2) / (d + 1))
            else:
                eta = mpmath.cospi(mpf(2 * k - 1) / (d + 1))
            z.append([mu_j, eta])
    return z


def create_sample_points_chebyshev(d: int, a=-1, b=1) -> List[object]:
    """Chebyshev nodes of the first kind, unisolvent up to degree d (MPMP.jl:186-191)."""
    a, b = mpf(a), mpf(b)
    return [(a + b) / 2 + (b - a) / 2 * mpmath.cos(mpf(2 * k - 1) / (2 * (d + 1)) * mp.pi)
            for k in range(1, d + 2)]


def create_sample_points_chebyshev_mod(d: int, a=-1, b=1) -> List[object]:
    """Chebyshev nodes divided by cos(pi/2(d+1)) (MPMP.jl:193-200)."""
    a, b = mpf(a), mpf(b)
    s = mpmath.cos(mp.pi / (2 * (d + 1)))
    return [(a + b) / 2 + (b - a) / 2 * mpmath.cos(mpf(2 * k - 1) / (2 * (d + 1)) * mp.pi) / s
            for k in range(1, d + 2)]


def create_sample_points_3d(d: int, pairs=((1, 3), (3, 2), (2, 1))) -> List[List[object]]:
    """Padua x Chebyshev points in 3 variables (MPMP.jl:122-145)."""
    pad = create_sample_points_2d(d)
    pad_div = [pad[0::3], pad[1::3], pad[2::3]]
    ch = create_sample_points_chebyshev(d + 2)
    cheb_div = [ch[0::3], ch[1::3], ch[2::3]]
    out = []
    for p1i, p2i in pairs:
        for p1 in pad_div[p1i - 1]:
            for p2 in cheb_div[p2i - 1]:
                out.append(list(p1) + [p2])
    return out[: (d + 1) * (d + 2) * (d + 3) // 6]


def points_X_general(n: int, d: int) -> List[List[object]]:
    """Recursive Padua/Chebyshev extension (MPMP.jl:147-170)."""
    if n == 2:
        return create_sample_points_2d(d)
    prev = points_X_general(n - 1, d)
    cheb = create_sample_points_chebyshev(d + n - 1)
    X_div = [prev[i::n] for i in range(n)]
    cheb_div = [cheb[i::n] for i in range(n)]
    out = []
    for i in range(1, n + 1):
        j = n if i == 1 else i - 1
        for p1 in X_div[i - 1]:
            for p2 in cheb_div[j - 1]:
                out.append(list(p1) + [p2])
    return out[: math.comb(n + d, d)]


def create_sample_points_1d(d: int) -> List[object]:
    """Rescaled-Laguerre points of Simmons-Duffin (MPMP.jl:173-182)."""
    const = -mpmath.sqrt(mp.pi) / (64 * (d + 1) * mpmath.log(3 - 2 * mpmath.sqrt(2)))
    return [const * (-1 + 4 * k) ** 2 for k in range(d + 1)]
