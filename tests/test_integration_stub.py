"""The reference-side ctypes binding shown in INTEGRATION.md section 2, executed against a fake
``libpfr`` on CPU: every batching mode of ``InnerState::solve`` (InnerState.h:164-308, modes 0-4 as
Sparse.py:245-282 selects them) must hand libpfr the right batch size, strides and right-hand-side
layout, and return the reference's output shape.  The fake solves each item densely from the
pointers it receives (host tensors stand in for device memory)."""
import ctypes as C
import os
import re

import numpy as np
import pytest
import scipy.sparse as sp

DOC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "INTEGRATION.md")


def _stub_source():
    txt = open(DOC).read()
    m = re.search(r"```python\n(# jax_plate/Sparse.py.*?)```", txt, re.S)
    assert m, "INTEGRATION.md section 2 stub not found"
    return m.group(1)


class _Fn:
    def __init__(self, f):
        self.f, self.argtypes, self.restype = f, None, None

    def __call__(self, *a):
        return self.f(*a)


class FakeLib:
    def __init__(self):
        self.pat = {}
        self.calls = []
        self.pfr_symbolic_create = _Fn(self._sym)
        self.pfr_solver_create = _Fn(self._solver)
        self.pfr_set_check = _Fn(lambda *a: 0)
        self.pfr_solve = _Fn(self._solve)
        self.pfr_solve_multi = _Fn(self._solve_multi)
        self.pfr_last_error = _Fn(lambda: b"")

    def _sym(self, n, nnz, cp, ri, opt, out):
        h = len(self.pat) + 1
        self.pat[h] = (n, np.ctypeslib.as_array(cp, (n + 1,)).copy(), np.ctypeslib.as_array(ri, (nnz,)).copy())
        out._obj.value = h
        return 0

    def _solver(self, sym, cp, ri, dev, mb, out):
        out._obj.value = sym.value
        return 0

    def _arr(self, ptr, count):
        return np.ctypeslib.as_array((C.c_double * (2 * count)).from_address(ptr)).view(np.complex128)

    def _one(self, h, d_ptr, ds, q, b_ptr, boff, x_ptr, xoff, transpose):
        n, cp, ri = self.pat[h]
        vals = self._arr(d_ptr + 16 * q * ds, cp[-1])
        A = sp.csc_matrix((vals, ri, cp), shape=(n, n)).toarray()
        b = self._arr(b_ptr + 16 * boff, n)
        x = self._arr(x_ptr + 16 * xoff, n)
        x[:] = np.linalg.solve(A.T if transpose else A, b)

    def _solve(self, s, batch, d, ds, b, bs, x, tr, flags, st):
        self.calls.append(("solve", batch, ds, bs))
        n = self.pat[s.value if hasattr(s, "value") else s][0]
        for q in range(batch):
            self._one(s.value, d, ds, q, b, q * bs, x, q * n, tr)
        return 0

    def _solve_multi(self, s, batch, nrhs, d, ds, b, bs, brs, x, xrs, tr, flags, st):
        self.calls.append(("multi", batch, nrhs, ds, bs, brs, xrs))
        n = self.pat[s.value][0]
        for r in range(nrhs):
            for q in range(batch):
                self._one(s.value, d, ds, q, b, r * brs + q * bs, x, r * xrs + q * n, tr)
        return 0


@pytest.fixture
def stub(monkeypatch):
    fake = FakeLib()
    monkeypatch.setattr(C, "CDLL", lambda path: fake)
    ns = {}
    exec(compile(_stub_source().replace('DEVICE = "cuda"', 'DEVICE = "cpu"'), "INTEGRATION.md", "exec"), ns)
    return ns, fake


@pytest.mark.parametrize("transpose", [False, True])
def test_all_batching_modes(stub, transpose):
    ns, fake = stub
    rng = np.random.default_rng(3)
    n, B, J = 9, 3, 2
    M = sp.random(n, n, density=0.4, random_state=1, format="csc") + sp.eye(n) * 4
    M = sp.csc_matrix(M)
    st = ns["SolverState"]()
    num = st.add_mat(M, M.T.tocsc(), np.stack(M.nonzero(), 1), np.arange(M.nnz))
    nnz = M.nnz
    data = rng.standard_normal((B, nnz)) + 1j * rng.standard_normal((B, nnz))
    c = M.tocoo()                                    # CSC order, like the data the solver receives
    data[:, c.row == c.col] += 6.0                   # keep every item well conditioned
    b = rng.standard_normal((J, B, n)) + 1j * rng.standard_normal((J, B, n))

    def dense(v):
        A = sp.csc_matrix((v, M.indices, M.indptr), shape=(n, n)).toarray()
        return A.T if transpose else A

    x0 = st.solve(data[0], b[0, 0], num, transpose, 0, 0)
    assert x0.shape == (n,) and np.allclose(x0, np.linalg.solve(dense(data[0]), b[0, 0]))
    x1 = st.solve(data, b[0, 0], num, transpose, 0, 1)
    assert x1.shape == (B, n) and all(np.allclose(x1[q], np.linalg.solve(dense(data[q]), b[0, 0])) for q in range(B))
    x2 = st.solve(data[0], b[0], num, transpose, 0, 2)
    assert x2.shape == (B, n) and all(np.allclose(x2[q], np.linalg.solve(dense(data[0]), b[0, q])) for q in range(B))
    x3 = st.solve(data, b[0], num, transpose, 0, 3)
    assert x3.shape == (B, n) and all(np.allclose(x3[q], np.linalg.solve(dense(data[q]), b[0, q])) for q in range(B))
    x4 = st.solve(data, b, num, transpose, 0, 4)
    assert x4.shape == (J, B, n)
    assert all(np.allclose(x4[j, q], np.linalg.solve(dense(data[q]), b[j, q])) for j in range(J) for q in range(B))
    assert [c[0] for c in fake.calls] == ["solve"] * 4 + ["multi"]
    assert fake.calls[1][1:] == (B, nnz, 0) and fake.calls[2][1:] == (B, 0, n)
