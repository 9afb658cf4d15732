"""Second, independent restatement of the code constructions in plain
Python/numpy (log/antilog field tables, closed-form Vandermonde), used only to
cross-check the C oracle in tests/test_oracle.py.  Test infrastructure.
"""
import numpy as np

# gf-complete / Jerasure default primitive polynomials (octal, as published)
POLY = {3: 0o13, 4: 0o23, 5: 0o45, 7: 0o211, 8: 0o435, 10: 0o2011, 11: 0o4005, 16: 0o210013}


class GF:
    def __init__(self, w):
        self.w = w
        n = (1 << w) - 1
        self.n = n
        self.exp = np.zeros(2 * n, dtype=np.int64)
        self.log = np.zeros(n + 1, dtype=np.int64)
        v = 1
        for i in range(n):
            self.exp[i] = self.exp[i + n] = v
            self.log[v] = i
            v <<= 1
            if v >> w:
                v ^= POLY[w]
        assert v == 1, "polynomial is not primitive"

    def mul(self, a, b):
        if a == 0 or b == 0:
            return 0
        return int(self.exp[self.log[a] + self.log[b]])

    def inv(self, a):
        return int(self.exp[(self.n - self.log[a]) % self.n])

    def matmul(self, A, B):
        R = np.zeros((A.shape[0], B.shape[1]), dtype=np.int64)
        for i in range(A.shape[0]):
            for j in range(B.shape[1]):
                acc = 0
                for l in range(A.shape[1]):
                    acc ^= self.mul(int(A[i, l]), int(B[l, j]))
                R[i, j] = acc
        return R

    def invert(self, A):
        n = A.shape[0]
        a = [list(map(int, r)) + [int(i == j) for j in range(n)] for i, r in enumerate(A)]
        for c in range(n):
            p = next(r for r in range(c, n) if a[r][c])
            a[c], a[p] = a[p], a[c]
            s = self.inv(a[c][c])
            a[c] = [self.mul(x, s) for x in a[c]]
            for r in range(n):
                if r != c and a[r][c]:
                    f = a[r][c]
                    a[r] = [x ^ self.mul(f, y) for x, y in zip(a[r], a[c])]
        return np.array([r[n:] for r in a], dtype=np.int64)


def vandermonde_closed_form(k, m, w):
    """C = normalise(V_bottom * V_top^-1) for the extended Vandermonde matrix:
    rows 0 = e0, i = [1, i, i^2, ...], last = e_{k-1}; coding row 0 and
    column 0 then scaled to ones (Jerasure's systematic distribution matrix)."""
    F = GF(w)
    rows = k + m
    V = np.zeros((rows, k), dtype=np.int64)
    V[0, 0] = 1
    V[rows - 1, k - 1] = 1
    for i in range(1, rows - 1):
        p = 1
        for j in range(k):
            V[i, j] = p
            p = F.mul(p, i)
    C = F.matmul(V[k:], F.invert(V[:k]))
    for j in range(k):  # columns: coding row 0 -> ones
        s = F.inv(int(C[0, j]))
        for i in range(m):
            C[i, j] = F.mul(int(C[i, j]), s)
    for i in range(1, m):  # rows: column 0 -> ones
        s = F.inv(int(C[i, 0]))
        for j in range(k):
            C[i, j] = F.mul(int(C[i, j]), s)
    return C


def bitmatrix_ones(F, e):
    ones = 0
    for _ in range(F.w):
        ones += bin(e).count("1")
        e = F.mul(e, 2)
    return ones


def cauchy_improved(k, m, w):
    """cauchy_original + cauchy_improve_coding_matrix (m > 2 path)."""
    F = GF(w)
    C = np.array([[F.inv(i ^ (m + j)) for j in range(k)] for i in range(m)], dtype=np.int64)
    for j in range(k):
        s = F.inv(int(C[0, j]))
        C[:, j] = [F.mul(int(x), s) for x in C[:, j]]
    for i in range(1, m):
        best = sum(bitmatrix_ones(F, int(x)) for x in C[i])
        pick = None
        for j in range(k):
            if C[i, j] == 1:
                continue
            s = F.inv(int(C[i, j]))
            tot = sum(bitmatrix_ones(F, F.mul(int(x), s)) for x in C[i])
            if tot < best:
                best, pick = tot, j
        if pick is not None:
            s = F.inv(int(C[i, pick]))
            C[i] = [F.mul(int(x), s) for x in C[i]]
    return C


def isal_cauchy1(k, m):
    F = GF(8)
    return np.array([[F.inv((i ^ j) & 0xFF) for j in range(k)] for i in range(k, k + m)],
                    dtype=np.int64)


def liberation(k, w):
    B = np.zeros((2 * w, k * w), dtype=np.int64)
    for j in range(k):
        for i in range(w):
            B[i, j * w + i] = 1
            B[w + i, j * w + (j + i) % w] = 1
        if j:
            y = j * (w - 1) // 2 % w
            B[w + y, j * w + (y + j - 1) % w] = 1
    return B


def to_bitmatrix(C, w):
    F = GF(w)
    m, k = C.shape
    B = np.zeros((m * w, k * w), dtype=np.int64)
    for i in range(m):
        for j in range(k):
            e = int(C[i, j])
            for x in range(w):
                for l in range(w):
                    B[i * w + l, j * w + x] = (e >> l) & 1
                e = F.mul(e, 2)
    return B


def rank_gf2(M):
    M = M.copy() % 2
    r = 0
    for c in range(M.shape[1]):
        piv = [i for i in range(r, M.shape[0]) if M[i, c]]
        if not piv:
            continue
        M[[r, piv[0]]] = M[[piv[0], r]]
        for i in range(M.shape[0]):
            if i != r and M[i, c]:
                M[i] ^= M[r]
        r += 1
    return r
