"""The laminate coefficients c = (A, B, D)(theta) and their Jacobian dc/dtheta in one forward-mode pass.

Host-side parameter math of every loss / FR evaluation (``Problem.getLossFunction``, ``getFRFunction``):
the material transforms of ``Material.py`` (reference ``Material.py:372-391, 455-482, 571-602, 743-764,
812-833``) restated on first-order jets -- value plus gradient over the n parameters -- so that one
evaluation gives c (18 complex) and J (18 x n complex) in numpy.  Through torch autograd the same 5-8
parameter transform builds and walks a graph of ~100 scalar ops per step (~1 ms of host time between
two GPU sweeps); ``coeffs18`` wraps the jet result in a custom autograd Function whose
backward is one product, ``grad_theta = Re(conj(grad_c) @ J)`` (torch's convention for complex outputs
of real inputs).  Formulas and operation order follow ``Material.py``; ``tests/test_abd_jet.py`` checks
values and Jacobians against the torch transforms for every material type.
"""
from __future__ import annotations

import numpy as np
import torch


class Jet:
    """a + grad . dtheta to first order (complex value, complex gradient over the parameters)."""

    __slots__ = ("v", "d")

    def __init__(self, v, d):
        self.v = complex(v)
        self.d = d

    @staticmethod
    def _lift(x, n):
        return x if isinstance(x, Jet) else Jet(x, np.zeros(n, dtype=np.complex128))

    def __add__(self, o):
        if isinstance(o, Jet):
            return Jet(self.v + o.v, self.d + o.d)
        return Jet(self.v + o, self.d)

    __radd__ = __add__

    def __neg__(self):
        return Jet(-self.v, -self.d)

    def __sub__(self, o):
        if isinstance(o, Jet):
            return Jet(self.v - o.v, self.d - o.d)
        return Jet(self.v - o, self.d)

    def __rsub__(self, o):
        return Jet(o - self.v, -self.d)

    def __mul__(self, o):
        if isinstance(o, Jet):
            return Jet(self.v * o.v, self.d * o.v + o.d * self.v)
        return Jet(self.v * o, self.d * o)

    __rmul__ = __mul__

    def __truediv__(self, o):
        if isinstance(o, Jet):
            q = self.v / o.v
            return Jet(q, (self.d - q * o.d) / o.v)
        return Jet(self.v / o, self.d / o)

    def __rtruediv__(self, o):
        q = o / self.v
        return Jet(q, -q / self.v * self.d)

    def __pow__(self, k: int):
        return Jet(self.v ** k, k * self.v ** (k - 1) * self.d)


def _params(theta):
    t = np.asarray(theta, dtype=np.float64)
    n = t.size
    eye = np.eye(n, dtype=np.complex128)
    return [Jet(t[i], eye[i].copy()) for i in range(n)], n


def _cplx_loss(beta: Jet, n: int) -> Jet:
    """1 + i beta"""
    return Jet(1.0 + 1j * beta.v.real, 1j * beta.d)


def _isotropic(p, n, h):
    E, G, beta = p
    nu = E / (2.0 * G) - 1.0
    A = E * h / (1 - nu ** 2)
    D = A * h ** 2 / 12.0
    loss = _cplx_loss(beta, n)
    arr = [Jet._lift(v, n) * loss for v in (1.0, nu, 0.0, 1.0, 0.0, (1 - nu) / 2)]
    zero = [Jet(0.0, np.zeros(n, dtype=np.complex128)) for _ in range(6)]
    return [A * a for a in arr], zero, [D * a for a in arr]


def _orthotropic_core(E1, E2, G12, nu12, h):
    e_ratio = E2 / E1
    nu21 = e_ratio * nu12
    A11 = E1 * h / (1 - nu12 * nu21)
    A12 = nu21 * A11
    A22 = E2 / E1 * A11
    A66 = G12 * h
    D11 = E1 * h ** 3 / (12 * (1 - nu12 * nu21))
    D66 = G12 * h ** 3 / 12
    D12 = nu21 * D11
    D22 = D11 / e_ratio          # reference quirk (Material.py:475): D22/D11 = E1/E2
    return (A11, A12, 0.0, A22, 0.0, A66), (D11, D12, 0.0, D22, 0.0, D66)


def _orthotropic(p, n, h):
    E1, E2, G12, nu12, beta = p
    As, Ds = _orthotropic_core(E1, E2, G12, nu12, h)
    loss = _cplx_loss(beta, n)
    zero = [Jet(0.0, np.zeros(n, dtype=np.complex128)) for _ in range(6)]
    return [Jet._lift(a, n) * loss for a in As], zero, [Jet._lift(d, n) * loss for d in Ds]


def _orthotropic_d4(p, n, h):
    E1, E2, G12, nu12 = (p[i] * _cplx_loss(p[4 + i], n) for i in range(4))
    As, Ds = _orthotropic_core(E1, E2, G12, nu12, h)
    zero = [Jet(0.0, np.zeros(n, dtype=np.complex128)) for _ in range(6)]
    return [Jet._lift(a, n) for a in As], zero, [Jet._lift(d, n) for d in Ds]


def _sol_q(E1, E2, G12, nu12, n):
    den = 1 - E2 / E1 * nu12 ** 2
    zero = Jet(0.0, np.zeros(n, dtype=np.complex128))
    return [E1 / den, nu12 * E2 / den, zero, E2 / den, zero, G12]


def _laminate(q, beta, maps, is_mps, n):
    vals = np.array([x.v for x in q])
    ders = np.stack([x.d for x in q])              # (6, n)
    loss = _cplx_loss(beta, n)
    out = []
    for k, M in enumerate(maps):
        mv, md = M @ vals, M @ ders
        out.append([Jet(mv[r], md[r].copy()) * loss for r in range(6)])
    if is_mps:
        out[1] = [Jet(0.0, np.zeros(n, dtype=np.complex128)) for _ in range(6)]
    return out


def abd_and_jacobian(material, h: float, theta):
    """(c (18,) complex128, J (18, n) complex128): c = [A, B, D] of the material at theta, J = dc/dtheta."""
    from .Material import laminate_q_to_abd
    p, n = _params(theta)
    atype = material.atype
    if atype == "isotropic":
        A, B, D = _isotropic(p, n, h)
    elif atype == "orthotropic":
        A, B, D = _orthotropic(p, n, h)
    elif atype == "orthotropic_d4":
        A, B, D = _orthotropic_d4(p, n, h)
    elif atype in ("sol", "symm_sol"):
        key = (tuple(np.asarray(material.angles, dtype=np.float64).tolist()), float(h))
        cache = material.__dict__.setdefault("_abd_maps", {})
        if key not in cache:
            cache[key] = [np.asarray(m, dtype=np.float64) for m in laminate_q_to_abd(material.angles, h)]
        maps = cache[key]
        if atype == "sol":
            q = _sol_q(p[0], p[1], p[2], p[3], n)
            beta = p[4]
        else:
            q = _sol_q(p[0], p[0], p[1], p[2], n)
            beta = p[3]
        A, B, D = _laminate(q, beta, maps, material.is_mps, n)
    else:
        raise ValueError(f"no jet transform for material type {atype!r}")
    jets = list(A) + list(B) + list(D)
    return (np.array([x.v for x in jets], dtype=np.complex128),
            np.stack([np.asarray(x.d, dtype=np.complex128) for x in jets]))


def _cached_abd(material, h: float, theta: np.ndarray):
    """abd_and_jacobian memoised on the last call per material (a pure function of the material's type and laminate,
    h and theta): a loss + gradient loop re-evaluated at one theta -- a benchmark, a line search's repeated point,
    the fr and loss of one iterate -- skips the jet pass (~100-200 us of Python per evaluation)."""
    key = (material.atype, float(h), theta.tobytes(),
           tuple(np.asarray(getattr(material, "angles", ()), dtype=np.float64).ravel().tolist()),
           bool(getattr(material, "is_mps", False)))
    last = material.__dict__.get("_abd_last")
    if last is not None and last[0] == key:
        return last[1], last[2]
    c, J = abd_and_jacobian(material, h, theta)
    material.__dict__["_abd_last"] = (key, c, J)
    return c, J


class _Coeffs(torch.autograd.Function):
    """theta (real, n) -> c (18 complex): values and Jacobian from the jet pass; backward one product."""

    @staticmethod
    def forward(ctx, theta, material, h):
        c, J = _cached_abd(material, h, theta.detach().cpu().numpy().astype(np.float64))
        ctx.J = J
        return torch.from_numpy(c.copy())

    @staticmethod
    def backward(ctx, grad_c):
        g = grad_c.detach().cpu().numpy()
        return torch.from_numpy(np.real(np.conj(g) @ ctx.J)).to(torch.float64), None, None


def coeffs18(material, h: float, theta: torch.Tensor) -> torch.Tensor:
    """c(theta) as a complex128 tensor of 18, differentiable in theta (float64, CPU)."""
    return _Coeffs.apply(theta, material, h)
