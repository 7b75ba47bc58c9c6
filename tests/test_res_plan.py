"""Which resident kernel every production split selects (gk_res_plan_query,
host-only: no GPU touched).

The single-GPU bench runs the w-only kernel (k_mgs_wres); the row-block splits
of the north-star grid over 2 / 4 / 8 GPUs, and config 4 (8192^2 over 8), give
each GPU a smaller slab and select the two-array kernels (k_mgs_res<12, L2>).
The -m gpu tests in tests/test_gpu_splits.py run exactly these variants with
two ranks on ONE GPU, each rank holding 128 workgroups (GK_TUNE_RES_SHARE 2)
and a slab chosen so that every workgroup carries the production split's
chunk load; this table pins that correspondence.
"""
import pytest

import gmres_amd as ga
from gmres_amd import _native


def _plan(N, R, share=1, hh=False, nt=-1):
    nl = max(n for _, n in ga.slab_partition(N, R))
    return ga.res_plan_query(N * nl, 256, share, hh, nt)


@pytest.mark.parametrize("hh", [False, True])
@pytest.mark.parametrize("N,R,variant,r2e,l2e,nt", [
    (4096, 1, "w-only", None, None, 1),    # the bench line (config 1), config 3 and 5
    (4096, 2, "w+column", 32, 0, 1),       # 8.4 M unknowns per GPU: w in registers, its column cached
    (4096, 4, "w+column", 16, 0, 1),       # 4.2 M (8 vs 10 B/unknown of k_mgs_res<12,4>)
    (4096, 8, "pairs", 8, 0, 0),           # 2.1 M (w+column ties at 8 B/unknown: the older kernel kept)
    (8192, 8, "w+column", 32, 0, 1),       # config 4: 8.4 M per GPU
    (1024, 1, "prefetch", 5, 0, 0),        # config 2
])
def test_production_splits(N, R, variant, r2e, l2e, nt, hh):
    p = _plan(N, R, hh=hh)
    assert p["variant"] == variant and p["G"] == 256
    assert p["l2e"] == (l2e if l2e is not None else (38 if hh else 39)) and p["nt"] == nt
    if variant == "w+column":  # 512 threads: 4 register + 19 LDS chunks of the column cached;
        # slabs of <= 16 chunks per thread: the 16-chunk kernel, the whole column in registers
        # (the MGS step caches 6 register chunks, the reflection chains 4)
        want = (16, 0, 0) if r2e <= 16 else ((4 if hh else 6), 19, 19 * 512 * 16)
        assert (p["r2"], p["l2"], p["lds"], p["wt"]) == want + (512,)
    if r2e is not None:
        assert p["r2e"] == r2e
    else:  # w-only: 89 + 39 (MGS-R) / 90 + 38 (reflection chains) chunks of 256 double2 -- the
        # whole 4096^2 slab (128 chunks per workgroup) on chip, nothing streamed
        assert p["r2e"] == (90 if hh else 89) and p["wt"] == 256
        assert p["nres2"] == N * N // 2, p


@pytest.mark.parametrize("R", [2, 4, 8])
@pytest.mark.parametrize("N,prod", [(1448, (4096, 8)), (2048, (4096, 4)), (2896, (4096, 2)), (4096, (4096, 1))])
def test_ranks_on_one_gpu_carry_the_production_load(N, prod, R):
    """R ranks x 256/R workgroups on one GPU (the -m gpu split tests): the same
    variant and the same chunks per workgroup as the production split on 256
    (the column load policy forced to the production split's, as the tests do)."""
    p = _plan(*prod)
    t = _plan(N, R, share=R, nt=p["nt"])
    assert t["G"] == 256 // R and p["G"] == 256 and t["nt"] == p["nt"]
    for k in ("variant", "r2e", "l2e"):
        assert t[k] == p[k], (k, t, p)
    dt = p["wt"]
    # resident double2 per workgroup agree within one chunk (ragged last chunk)
    assert abs(t["nres2"] / t["G"] - p["nres2"] / p["G"]) <= dt


def test_query_rejects_bad_arguments():
    buf = (_native.c_ll * len(_native.RES_INFO_KEYS))()
    assert _native.hip().gk_res_plan_query(1, 256, 1, 0, -1, 1, buf) == -1
    assert _native.hip().gk_res_plan_query(1 << 20, 0, 1, 0, -1, 1, buf) == -1


# The blocked-projection MGS step (GK_TUNE_RES_BLOCK = S, k_mgs_blk): the
# instantiation every production split selects -- register chunks of w per
# workgroup (512 threads; the w-only build 256 threads with LDS), the block cache
# per slot (r2 registers / l2 LDS), the dynamic LDS that fits 160 KiB.
BLOCKED = [
    # N, ranks, S -> (wt, r2e, l2e, r2, l2)
    (1024, 1, 2, (512, 4, 0, 4, 0)),
    (4096, 8, 2, (512, 8, 0, 8, 0)),
    (4096, 4, 2, (512, 16, 0, 7, 9)),
    (4096, 2, 2, (512, 32, 0, 1, 9)),
    (8192, 8, 2, (512, 32, 0, 1, 9)),
    (4096, 1, 2, (256, 90, 38, 0, 0)),
    (1024, 1, 4, (512, 4, 0, 4, 0)),
    (4096, 8, 4, (256, 16, 0, 16, 0)),  # one wave per SIMD: LDS left for the prefetch
    (4096, 4, 4, (512, 16, 0, 2, 4)),
    (4096, 2, 4, (512, 32, 0, 0, 4)),
    (4096, 1, 4, (256, 88, 38, 0, 0)),
]


@pytest.mark.parametrize("N,R,S,want", BLOCKED)
def test_blocked_plan_of_every_split(N, R, S, want):
    nl = max(n for _, n in ga.slab_partition(N, R))
    p = ga.res_plan_query(N * nl, 256, 1, False, -1, block=S)
    assert p["variant"] == "blocked" and p["blk"] == S and p["G"] == 256, p
    assert (p["wt"], p["r2e"], p["l2e"], p["r2"], p["l2"]) == want, p
    lw = 38 if p["wt"] == 256 and p["r2e"] > 32 else 0  # (the w-only build; not the one-wave S = 4 one)
    # LDS prefetch of small slabs: the next dot block's first chunks, capped at 96 KiB per
    # workgroup (GK_BLK_PFX_KB; profiles/r05/ab_blk_pfx_kb_r05ae.txt)
    chunks = {(512, 4): 4, (512, 8): 8, (256, 16): 8}.get((p["wt"], p["r2e"]), 0)
    pfx = min(chunks, 96 * 1024 // (S * p["wt"] * 16))
    assert p["lds"] == (lw + S * (p["l2"] + pfx)) * p["wt"] * 16 and p["lds"] + 5 * 1024 <= 160 * 1024, p
    # the whole slab is resident except the w-only S = 4 build's two streamed chunks
    assert p["nres2"] <= N * nl // 2


def test_blocked_plan_leaves_householder_strict():
    for S in (2, 4):
        p = ga.res_plan_query(4096 * 4096, 256, 1, True, -1, block=S)
        assert p["variant"] != "blocked" and p["blk"] == 1, p


def test_blocked_plan_rejects_other_blocks():
    buf = (_native.c_ll * len(_native.RES_INFO_KEYS))()
    assert _native.hip().gk_res_plan_query(1 << 20, 256, 1, 0, -1, 3, buf) == -1

