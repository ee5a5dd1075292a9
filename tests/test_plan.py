"""Host-side plan of the band kernel (C ABI nldsc_plan_band; no GPU): the window replay equals the
oracle's replay of the reference pointers, and the work items cover every block pair holding a
needed (SNP, neighbour) pair for the owned range."""
import numpy as np
import pytest

from conftest import load_set
from oracle import oracle as O


def needed_blocks(pos, passed, w, L, R, own):
    """{(I, J)} block pairs (I <= J) that hold some j in N(i) with i owned (row) or ..."""
    need = set()
    for i in range(len(pos)):
        if L[i] < 0 or not (own[0] <= i < own[1]):
            continue
        for k in range(L[i], R[i] + 1):
            if k != i and passed[k] and abs(pos[k] - pos[i]) <= w:
                a, b = sorted((i // 32, k // 32))
                need.add((a, b))
    return need


def covered(items):
    cov = set()
    for I, J0, nc, _ in items:
        assert I <= J0 and nc in (1, 2)
        for b in range(nc):
            cov.add((int(I), int(J0) + b))
    return cov


def check(pos, passed, w, own=None, max_nc=1):
    from nldsc_amd import _lib
    n = len(pos)
    own = (0, n) if own is None else own
    L, R, items = _lib.plan_band(pos, passed.astype(np.uint8), w, own=own, max_nc=max_nc)
    Lp, Rp = O.replay_windows(pos, passed, w)
    np.testing.assert_array_equal(L, Lp)
    np.testing.assert_array_equal(R[L >= 0], Rp[Lp >= 0])
    nblk = (n + 31) // 32
    assert all(J0 + nc <= nblk for _, J0, nc, _ in items)
    miss = needed_blocks(pos, passed, w, L, R, own) - covered(items)
    assert not miss, sorted(miss)[:10]
    return items


@pytest.mark.parametrize("name", ["n1000", "n1003", "allmiss"])
def test_plan_covers_golden_sets(name):
    _, pos, meta, orc, _ = load_set(name)
    passed = (pos >= 0) & ~(orc["maf"] <= meta["maf"])
    for nc in (1, 2):
        check(pos, passed, meta["ld_wind"], max_nc=nc)
    M = meta["n_snp"]
    for own in ((0, 100), (M // 3, 2 * M // 3), (M - 50, M)):
        check(pos, passed, meta["ld_wind"], own=own)


@pytest.mark.parametrize("seed", range(6))
def test_plan_covers_random_and_unsorted(seed):
    rng = np.random.default_rng(seed)
    n = int(rng.integers(1, 400))
    pos = np.cumsum(rng.exponential(0.02, n))
    if seed % 2:  # unsorted: the reference's pointer semantics, the plan falls back to R as bound
        pos = pos[rng.permutation(n)]
    pos[rng.random(n) < 0.05] = -1.0
    passed = (pos >= 0) & (rng.random(n) > 0.1)
    w = float(rng.choice([0.01, 0.3, 5.0]))
    check(pos, passed, w, max_nc=1 + seed % 2)
    a = int(rng.integers(0, n))
    check(pos, passed, w, own=(a, min(n, a + 57)))


def test_plan_is_tight_on_c3_geometry():
    """chr1-like C3 positions (80 000 SNPs over 280 cM, 1 cM): about 10.4 column blocks per row block
    (the geometric minimum for 32-SNP blocks; the reference's loose cache bound R would give 12.5)."""
    from nldsc_amd import _lib
    rng = np.random.default_rng(7)
    M = 80_000
    rng.uniform(0.02, 0.5, size=M)
    pos = np.round(np.cumsum(rng.exponential(280.0 / M, size=M)), 6)
    _, _, items = _lib.plan_band(pos, np.ones(M, np.uint8), 1.0)
    assert len(items) / ((M + 31) // 32) < 10.6


def left_pointers_from_all_pass(pos, passed, A):
    """The rule left_pointer_kernel applies (sorted positions): L_j = first used passing SNP in
    [A_j, j), else j; -1 where A_j < 0 or j fails MAF."""
    used = pos >= 0
    L = np.full(len(pos), -1)
    for j in range(len(pos)):
        if A[j] < 0 or not passed[j]:
            continue
        i = A[j]
        while i < j and not (passed[i] and used[i]):
            i += 1
        L[j] = i
    return L


@pytest.mark.parametrize("seed", range(40))
def test_left_pointers_from_all_pass_replay(seed):
    """Sorted positions: the sequential replay's (L, R) equal (rule above, all-pass R) — ties, unused SNPs
    (pos < 0, including the lagging right pointer they cause), w = 0 and heavy MAF failure included."""
    rng = np.random.default_rng(500 + seed)
    n = int(rng.integers(1, 300))
    pos = np.cumsum(rng.exponential(rng.choice([0.005, 0.05, 0.5]), n))
    if seed % 3 == 0:
        pos = np.round(pos, 1)
    pos[rng.random(n) < rng.choice([0, 0.05, 0.3, 0.7])] = -1.0
    passed = rng.random(n) > rng.choice([0, 0.1, 0.6])
    w = float(rng.choice([0.0, 0.01, 0.1, 1.0, 10.0]))
    L, R = O.replay_windows(pos, passed, w)
    A, Ra = O.replay_windows(pos, np.ones(n, bool), w)
    np.testing.assert_array_equal(L, left_pointers_from_all_pass(pos, passed, A))
    np.testing.assert_array_equal(R[L >= 0], Ra[L >= 0])


def gpu_schedule_restated(pos, w, own):
    """numpy restatement of the GPU schedule kernels (ld_kernels.hip plan_*): window edges E by the exact
    predicate, all-pass left pointers A, right pointers R = min(n-1, j + running max(E_k - k)), and the
    per-row-block useful offset ranges -> the set of block pairs."""
    n = len(pos)
    E = np.array([next((k for k in range(j + 1, n) if pos[k] - pos[j] > w), n) for j in range(n)])
    A = np.array([next(k for k in range(j + 1) if pos[j] - pos[k] <= w) for j in range(n)])
    R = np.minimum(n - 1, np.arange(n) + np.maximum.accumulate(E - np.arange(n)))
    nblk = (n + 31) // 32
    ob0, ob1 = own[0] // 32, (own[1] - 1) // 32
    pairs = set()
    for I in range(A[own[0]] // 32, nblk):
        if I * 32 >= own[1]:
            break
        jmax = min(nblk - 1, (E[min(n, 32 * I + 32) - 1] - 1) // 32)
        own_row = ob0 <= I <= ob1
        J0, J1 = (I, jmax) if own_row else (max(I, ob0), min(jmax, ob1))
        pairs |= {(I, J) for J in range(J0, J1 + 1)}
    return A, R, pairs


@pytest.mark.parametrize("seed", range(5))
def test_gpu_schedule_formulas_match_host_replay(seed):
    """The closed forms the GPU schedule uses for non-negative sorted positions reproduce the host replay of
    ChunkwiseReader (all-pass left/right pointers) and cover every needed block pair; the host plan's own
    items are a subset of them (the GPU bound uses the exact |dpos| <= w predicate)."""
    from nldsc_amd import _lib
    rng = np.random.default_rng(900 + seed)
    n = int(rng.integers(40, 700))
    pos = np.cumsum(rng.exponential(0.02, n))
    if seed % 2:
        pos = np.round(pos, 2)  # ties
    w = float(rng.choice([0.1, 0.25, 1.0]))
    passed = np.ones(n, bool)
    for own in ((0, n), (n // 4, n // 2), (n - 1, n)):
        A, R, pairs = gpu_schedule_restated(pos, w, own)
        L, Rh, items = _lib.plan_band(pos, passed.astype(np.uint8), w, own=own, max_nc=1)
        np.testing.assert_array_equal(A, L)
        np.testing.assert_array_equal(R, Rh)
        assert covered(items) <= pairs
        assert not (needed_blocks(pos, passed, w, L, Rh, own) - pairs)
