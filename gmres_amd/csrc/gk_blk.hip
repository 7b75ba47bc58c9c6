// gk_blk.hip -- the blocked-projection MGS-R step (gk_blk.hpp): one all-gather
// per block of S projections instead of one per projection.  Opt-in
// (GK_TUNE_RES_BLOCK); the default stays the strict MGS-R step of
// gmres_mgsr.f90:341-360 (k_mgs_wres / k_mgs_wpc / k_mgs_res, gk_kernels.hpp).
#include <hip/hip_runtime.h>

#include <atomic>

#include "gk_blk.hpp"
#include "gk_res.hpp"

namespace gk {

namespace {

// Block b of a sweep of step j (0-based columns): b = 0 -> {0}; b >= 1 -> the
// columns 1 + (b-1)S .. min(bS, j-1).
__device__ __forceinline__ int blk_lo(int b, int S) { return b == 0 ? 0 : 1 + (b - 1) * S; }
__device__ __forceinline__ int blk_n(int b, int S, int j) { return b == 0 ? 1 : min(S, j - blk_lo(b, S)); }

// a wave-uniform double into scalar registers
__device__ __forceinline__ double uniform(double v) {
    const long long b = __double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)b);
    const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(b >> 32));
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

#ifndef GK_BLK_POLL_SLEEP
#define GK_BLK_POLL_SLEEP 16
#endif
constexpr int BLK_POLL_SLEEP = GK_BLK_POLL_SLEEP;
#ifndef GK_BLK_REV2
#define GK_BLK_REV2 1
#endif
constexpr bool BLK_REV2 = GK_BLK_REV2 != 0;  // the second sweep's blocks in reverse order (A/B knob)
#ifndef GK_BLK_DOT_NT
#define GK_BLK_DOT_NT 0
#endif
// 1: the dot columns of cached chunks non-temporal (they are held on chip from then
// on); 0: the default policy, so a column read again within the Infinity Cache's
// reach (the reversed second sweep, the next step's first sweep) is a hit (A/B knob)
constexpr bool BLK_DOT_NT = GK_BLK_DOT_NT != 0;
#ifndef GK_BLK_PF_SPLIT
#define GK_BLK_PF_SPLIT 1
#endif
// the strict step on this kernel (S = 1, GK_TUNE_RES_PF): the prefetch during an all-gather
// from the waves that do not poll it, so the poll -- and on N ranks a rank-total pusher's push --
// does not queue behind it (4-rank rehearsal 935 -> 968 it/s, single GPU +1 %:
// profiles/r05/ab_strict_pf_split_r05aq.txt); blocks of 2 / 4 keep every wave its own
// elements (a wash there: ab_blk_pf_split_r05ak.txt)
constexpr bool BLK_PF_SPLIT = GK_BLK_PF_SPLIT != 0;
#ifndef GK_BLK_WB_LDS
#define GK_BLK_WB_LDS 2
#endif
// batch of the LDS part of w (its loop is not unrolled: a deeper batch spilled the
// one-wave build, whose registers hold 88 chunks of w)
constexpr int BLK_WB_LDS = GK_BLK_WB_LDS;
// Dot columns not cached on chip are read with the default policy: they come back
// as the next pass's AXPY columns.  (At 4096^2 the S dot columns of a pass outgrow
// the 256 MiB Infinity Cache; reading the second slot non-temporal -- wholly, past
// chunk 64 or past the 90 register chunks -- measured slower still: 196.4 / 196.1 /
// 202.1 vs 210.6 it/s, profiles/r05/ab_blk_qdef_4096_r05d.txt.)

}  // namespace

// --------------------------------------------------------------------------
// k_mgs_blk: one persistent launch per Arnoldi step (one workgroup per CU), the
// resident layout of the strict kernels: w of RW chunks per thread in registers
// and LW more in LDS (the rest streams through HBM); the column cache keeps the
// S columns of the block the next pass subtracts -- RX chunks per column in
// registers, LX in LDS, for register chunks of w only.  A pass reads the S dot
// columns of the NEXT block once (8 B per unknown per projection where cached;
// past the cache the AXPY columns are read again, the dot columns then with the
// default policy so that re-read is an Infinity-Cache hit), subtracts the current
// block's columns with the h it holds, takes the dots and the Gram terms with the
// block's last column, and closes with ONE multi-value all-gather (res_publish_v /
// res_collect_v: value v on wave v).  Thread 0 then forms the next block's h by the recurrence of
// gk_blk.hpp.  The last pass closes with ||w||^2; V(:,j+1) = w / ||w|| and
// H(1:j+1, j) as in the strict kernels.
//
// Slots: every block is held in S slots, its r real columns in the LAST r (so the
// block's last column -- the newest column of the step, in the block that holds it
// -- is always slot S-1) and dummies in front: a dummy subtracts with h = 0 (exact:
// w - 0 x = w) and addresses the block's first real column (its loads hit the
// caches: no extra HBM bytes), so the unrolled pass has no per-column branches.
// TCH > 0: the waves not busy with the all-gather touch the first TCH chunks of
// the following pass's last dot column into L2 (k_mgs_wres's paced touch).
// PFX > 0 (small slabs, whose pass is one memory latency): the dot block of the
// NEXT pass is loaded for chunks 0 .. PFX-1 straight into LDS (global_load_lds,
// no VGPRs) before each all-gather, so its loads overlap the all-gather instead of
// opening the next pass (the strict small-slab kernel's prefetch, k_mgs_res PF).
// --------------------------------------------------------------------------
typedef __attribute__((address_space(3))) void lds_void_t;
template <int RW, int LW, int RX, int LX, int S, int WBT, int TCH, int NT, int PFX = 0>
__global__ __launch_bounds__(NT, 1) void k_mgs_blk(ResArgs a) {
    static_assert(S >= 1 && S <= RES_SMAX, "blocks of 1..RES_SMAX projections");
    static_assert(RX + LX <= RW, "the column cache covers register chunks of w only");
    static_assert(PFX <= RX && (PFX == 0 || (LW == 0 && LX == 0)), "the prefetch covers register-cached chunks");
    constexpr int NW = NT / 64, KM = 2 * S - 1;
    extern __shared__ double2 lsh[];
    double2 *__restrict__ lw = lsh;            // [LW][NT]: w beyond the registers
    double2 *__restrict__ lx = lsh + LW * NT;  // [S][LX][NT]: cached columns, chunks RX .. RX+LX-1
    double2 *__restrict__ lpf = lx + S * LX * NT;  // [S][PFX][NT]: the next pass's dot block (PFX > 0)
    __shared__ double sm[KM][NW];
    __shared__ double bc[KM];
    __shared__ double hv[S];      // h of the block the next pass subtracts, by slot (0: dummy)
    __shared__ double gbuf[(RES_SMAX - 1) * RES_SMAX];  // Gram table rows of the block a pass dots with
    __shared__ int okf, xdone;
    __shared__ double hsh[RHMAX + 1];
    const int t = threadIdx.x, wv = t >> 6, lane = t & 63;
    const int j = a.j;
    const int nb1 = blk_sweep(j, S), P = 2 * nb1;
    // the block pass p subtracts: the first sweep in column order, the second (REV2)
    // in reverse -- its first block is the one the first sweep ended with (still on
    // chip), and the columns read last come back first (Infinity-Cache hits at the
    // split loads); in exact arithmetic the second sweep's h are all 0 in any order
    // (S = 1 is strict MGS-R: both sweeps in the reference's column order)
    auto blk_of = [&](int p) { return p < nb1 ? p : (BLK_REV2 && S > 1 ? 2 * nb1 - 1 - p : p - nb1); };
    const i64 n2 = a.n >> 1, ld2 = a.ld >> 1;
    const i64 nch = a.nres2 / NT;
    const i64 c0 = (i64)blockIdx.x * a.r2e, cend = c0 + a.r2e < nch ? c0 + a.r2e : nch;
    const i64 l0 = (i64)gridDim.x * a.r2e + (i64)blockIdx.x * a.l2e, lend = l0 + a.l2e < nch ? l0 + a.l2e : nch;
    const double2 *__restrict__ V2 = reinterpret_cast<const double2 *>(a.V);
    double2 *__restrict__ W2 = reinterpret_cast<double2 *>(a.w);
    ResClock clk;
    clk.start(a.stamps);
    const i64 sstride = (i64)gridDim.x * NT;
    // the chunk range as opaque copies at each use: otherwise the compiler hoists RW
    // chunk predicates and offsets out of the pass loop into scalar registers, which
    // spill into VGPR lanes beside the register-held w
    auto range = [&](int &b, int &e) {
        b = (int)c0;
        e = (int)cend;
        asm volatile("" : "+s"(b), "+s"(e));
    };
    const unsigned vo = (unsigned)t * 16u;  // this lane's byte offset in a chunk
    auto at = [&](const double2 *base, int c) {  // element t of chunk c of a column
        return reinterpret_cast<const double2 *>(reinterpret_cast<const char *>(base + (i64)c * NT) + vo);
    };
    // the dot block (id, rd) of the next pass, chunks < PFX, into lpf by global_load_lds
    // (dummy slots load the block's first real column: finite values for h = 0)
    // kpoll < NW (during an all-gather whose K values are polled by waves 0 .. K-1, on N
    // ranks the rank-total pushers among them): the waves kpoll .. NW-1 load every wave's
    // elements, so the polls -- and a pusher's push -- do not wait, in their wave's vmcnt
    // order, for the prefetch to land; the barrier after the all-gather hands the LDS over
    auto prefetch = [&](int id, int rd, int kpoll) {
        if constexpr (PFX > 0) {
            int cb, ce;
            range(cb, ce);
            const int nd = NW - kpoll, wd = wv - kpoll;
            if (kpoll >= NW) {
#pragma unroll
                for (int d = 0; d < S; ++d) {
                    const int qd = d - (S - rd);
                    const double2 *D = V2 + (i64)(id + (qd > 0 ? qd : 0)) * ld2;
#pragma unroll
                    for (int k = 0; k < PFX; ++k)
                        if (cb + k < ce)
                            __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(at(D, cb + k)),
                                                             (lds_void_t *)(lpf + (d * PFX + k) * NT + (t & ~63)), 16, 0,
                                                             0);
                }
            } else if (wd >= 0) {
                for (int g = wd; g < NW; g += nd)  // element group g (64 elements) of every chunk
#pragma unroll
                    for (int d = 0; d < S; ++d) {
                        const int qd = d - (S - rd);
                        const double2 *D = V2 + (i64)(id + (qd > 0 ? qd : 0)) * ld2 + g * 64;
#pragma unroll
                        for (int k = 0; k < PFX; ++k)
                            if (cb + k < ce)
                                __builtin_amdgcn_global_load_lds(
                                    reinterpret_cast<const void *>(reinterpret_cast<const char *>(D + (i64)(cb + k) * NT) +
                                                                   lane * 16),
                                    (lds_void_t *)(lpf + (d * PFX + k) * NT + g * 64), 16, 0, 0);
                    }
            }
        }
    };
    double2 wr[RW], xc[S][RX > 0 ? RX : 1];
    // w, and V(:,1) -- block 0, subtracted by pass 0 from slot S-1 -- into the cache
    // (the dummy slots zero)
    {
        int cb, ce;
        range(cb, ce);
#pragma unroll
        for (int k = 0; k < RW; ++k) wr[k] = (cb + k < ce) ? *at(W2, cb + k) : double2{0.0, 0.0};
#pragma unroll
        for (int k = 0; k < RX; ++k) {
#pragma unroll
            for (int s = 0; s < S - 1; ++s) xc[s][k] = double2{0.0, 0.0};
            xc[S - 1][k] = (cb + k < ce) ? ldv<true>(at(V2, cb + k)) : double2{0.0, 0.0};
        }
        for (int k = 0; k < LX; ++k)
            if (cb + RX + k < ce) {
                for (int s = 0; s < S - 1; ++s) lx[(s * LX + k) * NT + t] = double2{0.0, 0.0};
                lx[((S - 1) * LX + k) * NT + t] = ldv<true>(at(V2, cb + RX + k));
            }
    }
    for (int k = 0; k < LW; ++k)
        if (l0 + k < lend) lw[k * NT + t] = W2[(l0 + k) * NT + t];
    prefetch(blk_lo(blk_of(1), S), blk_n(blk_of(1), S, j), NW);  // pass 0's dot block
    // h of block 0 = <w, V(:,1)>: the operator launch's partial slab (on N ranks
    // its rank hop here, res_pin_fold)
    double h;
    {
        if constexpr (PFX > 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        double s = 0.0;
        for (int k = t; k < a.npin; k += NT) s += a.pin[k];
        s = wave_sum(s);
        if (lane == 0) sm[0][wv] = s;
        __syncthreads();
        h = sm[0][0];
#pragma unroll
        for (int w = 1; w < NW; ++w) h += sm[0][w];
        __syncthreads();
    }
    bool ok = res_pin_fold(a, h, bc, &okf);
    if (t == 0) {
#pragma unroll
        for (int s = 0; s < S - 1; ++s) hv[s] = 0.0;
        hv[S - 1] = h;
        if (blockIdx.x == 0) hsh[0] = h;  // H(1, j), first sweep
    }
    __syncthreads();

    // One pass: subtract block (ia, ra) with hc, then the S dots with block (id, rd)
    // and the Gram terms <slot l, slot S-1> -- or, nrm (the last pass), ||w||^2 into
    // acc[0] by a uniform select (the dot columns then address the subtracted block:
    // one instantiation of the unrolled pass -- two inlined kinds spilled w)
    double acc[KM];
    auto pass = [&](bool nrm, int ia, int ra, int id, int rd) {
        const double2 *A[S], *D[S];
        double hc[S];  // uniform: scalar registers
#pragma unroll
        for (int s = 0; s < S; ++s) {
            const int qa = s - (S - ra), qd = s - (S - rd);
            A[s] = V2 + (i64)(ia + (qa > 0 ? qa : 0)) * ld2;
            D[s] = nrm ? A[s] : V2 + (i64)(id + (qd > 0 ? qd : 0)) * ld2;
            hc[s] = qa >= 0 ? uniform(hv[s]) : 0.0;
        }
#pragma unroll
        for (int e = 0; e < KM; ++e) acc[e] = 0.0;
        // the closing reductions of one element pair of w (after the AXPYs)
        auto red = [&](const double2 &x, const double2 (&b)[S]) {
            const double2 y0 = nrm ? x : b[0];
            acc[0] = acc[0] + x.x * y0.x;
            acc[0] = acc[0] + x.y * y0.y;
#pragma unroll
            for (int d = 1; d < S; ++d) {
                acc[d] = acc[d] + x.x * b[d].x;
                acc[d] = acc[d] + x.y * b[d].y;
            }
#pragma unroll
            for (int l = 0; l < S - 1; ++l) {
                acc[S + l] = acc[S + l] + b[l].x * b[S - 1].x;
                acc[S + l] = acc[S + l] + b[l].y * b[S - 1].y;
            }
        };
        int cb, ce;
        range(cb, ce);
        // register chunks of w, batches of WBT
#pragma unroll
        for (int k0 = 0; k0 < RW; k0 += WBT) {
            double2 bv[WBT][S], av[WBT][S];
#pragma unroll
            for (int u = 0; u < WBT; ++u) {
                const int k = k0 + u;
                if (k < RW && cb + k < ce) {
#pragma unroll
                    for (int d = 0; d < S; ++d) {
                        if (k < PFX)  // (the norm pass reads a stale but finite block here: unused)
                            bv[u][d] = lpf[(d * PFX + (k < PFX ? k : 0)) * NT + t];
                        else if (k < RX + LX && BLK_DOT_NT)
                            bv[u][d] = ldv<true>(at(D[d], cb + k));
                        else
                            bv[u][d] = ldv<false>(at(D[d], cb + k));
                    }
                    if (k >= RX + LX) {
#pragma unroll
                        for (int s = 0; s < S; ++s) av[u][s] = ldv<true>(at(A[s], cb + k));
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < WBT; ++u) {
                const int k = k0 + u;
                if (k < RW && cb + k < ce) {
#pragma unroll
                    for (int s = 0; s < S; ++s) {
                        double2 x;
                        if (k < RX)
                            x = xc[s][k < RX ? k : 0];
                        else if (k < RX + LX)
                            x = lx[(s * LX + (k - RX)) * NT + t];
                        else
                            x = av[u][s];
                        wr[k].x = wr[k].x - hc[s] * x.x;
                        wr[k].y = wr[k].y - hc[s] * x.y;
                    }
                    red(wr[k], bv[u]);
                    if (k < RX + LX) {
#pragma unroll
                        for (int d = 0; d < S; ++d) {
                            if (k < RX)
                                xc[d][k < RX ? k : 0] = bv[u][d];
                            else
                                lx[(d * LX + (k - RX)) * NT + t] = bv[u][d];
                        }
                    }
                }
            }
        }
        // LDS chunks of w: both blocks' columns from memory
        constexpr int WBL = WBT < BLK_WB_LDS ? WBT : BLK_WB_LDS;
        for (int k0 = 0; k0 < LW; k0 += WBL) {
            double2 bv[WBL][S], av[WBL][S];
#pragma unroll
            for (int u = 0; u < WBL; ++u) {
                const i64 c = l0 + k0 + u;
                if (k0 + u < LW && c < lend) {
#pragma unroll
                    for (int d = 0; d < S; ++d)
                        bv[u][d] = ldv<false>(at(D[d], (int)c));
#pragma unroll
                    for (int s = 0; s < S; ++s) av[u][s] = ldv<true>(at(A[s], (int)c));
                }
            }
#pragma unroll
            for (int u = 0; u < WBL; ++u) {
                const int k = k0 + u;
                if (k < LW && l0 + k < lend) {
                    double2 x = lw[k * NT + t];
#pragma unroll
                    for (int s = 0; s < S; ++s) {
                        x.x = x.x - hc[s] * av[u][s].x;
                        x.y = x.y - hc[s] * av[u][s].y;
                    }
                    lw[k * NT + t] = x;
                    red(x, bv[u]);
                }
            }
        }
        // streamed part: w and every column from HBM, one element pair at a time
        for (i64 e = a.nres2 + (i64)res_stream_wg() * NT + t; e < n2; e += sstride) {
            double2 x = W2[e], bv[S];
#pragma unroll
            for (int s = 0; s < S; ++s) {
                const double2 v = ldv<true>(A[s] + e);
                x.x = x.x - hc[s] * v.x;
                x.y = x.y - hc[s] * v.y;
            }
            W2[e] = x;
#pragma unroll
            for (int d = 0; d < S; ++d) bv[d] = ldv<false>(D[d] + e);
            red(x, bv);
        }
        if ((a.n & 1) && blockIdx.x == gridDim.x - 1 && t == 0) {  // odd-length tail element
            const i64 e = a.n - 1;
            double x = a.w[e];
#pragma unroll
            for (int s = 0; s < S; ++s) x = x - hc[s] * reinterpret_cast<const double *>(A[s])[e];
            a.w[e] = x;
            double2 bt[S];
#pragma unroll
            for (int d = 0; d < S; ++d) bt[d] = double2{reinterpret_cast<const double *>(D[d])[e], 0.0};
            red(double2{x, 0.0}, bt);
        }
    };

    int xi = 0;
    int touch_sink = 0;
    for (int p = 0; p < P && ok; ++p) {
        const int ba = blk_of(p), ia = blk_lo(ba, S), ra = blk_n(ba, S, j);
        const bool last = p == P - 1;
        const int bd = blk_of(p + 1), id = blk_lo(bd, S), rd = last ? 1 : blk_n(bd, S, j);
        const bool gram = !last && bd == nb1 - 1 && rd >= 2;  // the block of the newest column j-1
        // the stored Gram terms of block bd (the newest column's come with this
        // all-gather): rows id+1 .. id+S-1 of the table, straight into LDS by wave 0
        // (global_load_lds: no VGPRs, no wait) for thread 0's recurrence after the
        // all-gather -- gbuf[(k-1) * RES_SMAX + d] = <V(id+k-d), V(id+k)>
        if (!last && t < 2 * (S - 1))
            __builtin_amdgcn_global_load_lds(
                reinterpret_cast<const void *>(a.gm + (i64)(id + 1) * RES_SMAX + 2 * t), (lds_void_t *)gbuf, 16, 0, 0);
        pass(last, ia, ra, id, rd);
        // the all-gather: value v = the dot of real column v of block bd (slot S-rd+v),
        // then value rd + l = the Gram term <slot S-rd+l, slot S-1>
        clk.passed(a.stamps);
        const int K = last ? 1 : rd + (gram ? rd - 1 : 0);
#pragma unroll
        for (int e = 0; e < KM; ++e) {
            int v = -1;
            if (last)
                v = e == 0 ? 0 : -1;
            else if (e < S)
                v = e >= S - rd ? e - (S - rd) : -1;
            else if (gram)
                v = (e - S) >= S - rd ? rd + (e - S) - (S - rd) : -1;
            if (v >= 0) {
                const double r = wave_sum(acc[e]);
                if (lane == 0) sm[v][wv] = r;
            }
        }
        if (t == 0) {
            okf = 1;
            xdone = 0;
        }
        __syncthreads();
        // value v on wave v (and v + NW, ... when a block has more values than waves):
        // publish first, then (PFX) the next pass's dot block -- its loads queue behind
        // the publish, not in front of it -- then collect
        const int vend = KM <= NW ? (wv < K ? wv + 1 : 0) : K;
        for (int v = wv; v < vend; v += NW) {
            double s = sm[v][0];
#pragma unroll
            for (int w = 1; w < NW; ++w) s += sm[v][w];
            if (a.trace != nullptr && t == 0 && xi < RES_TRACE_X)  // (gk_profile_res_trace)
                a.trace[((i64)blockIdx.x * RES_TRACE_X + xi) * 2] = wall_clock64();
            res_publish_v(a, xi, v, s);
        }
        if (p + 2 < P) {  // the next pass reduces dots: its block's loads overlap this all-gather
            const int b2 = blk_of(p + 2);
            prefetch(blk_lo(b2, S), blk_n(b2, S, j), BLK_PF_SPLIT && S == 1 ? K : NW);
        }
        for (int v = wv; v < vend; v += NW) {
            double out = 0.0;
            const bool okv = res_collect_v<BLK_POLL_SLEEP>(a, xi, v, &out);
            if (lane == 0) {
                bc[v] = out;
                if (!okv) okf = 0;
            }
            if (a.trace != nullptr && t == 0 && xi < RES_TRACE_X)
                a.trace[((i64)blockIdx.x * RES_TRACE_X + xi) * 2 + 1] = wall_clock64();
        }
        if (wv < K && lane == 0) atomicAdd(&xdone, 1);
        if constexpr (TCH > 0) {
            // the first TCH chunks of the following pass's last dot column, one dword per
            // 128-B line, paced, until every all-gather wave holds its total
            const int kw = K < NW ? K : NW;
            if (wv >= kw && p + 2 < P) {
                const int b2 = blk_of(p + 2);
                const int tcol = blk_lo(b2, S) + blk_n(b2, S, j) - 1;
                const char *base = reinterpret_cast<const char *>(V2 + (i64)tcol * ld2 + c0 * NT);
                const i64 nc = cend - c0 < TCH ? (cend - c0 > 0 ? cend - c0 : 0) : TCH;
                for (i64 l = t - 64 * kw; l < 32 * nc; l += NT - 64 * kw) {
                    if (*(volatile int *)&xdone >= kw) break;  // wave-uniform: one LDS word
                    asm volatile("global_load_dword %0, %1, off" : "+v"(touch_sink) : "v"(base + l * 128) : "memory");
                    __builtin_amdgcn_s_sleep(24);
                }
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's LDS-DMA (prefetch, Gram rows) landed
        __syncthreads();
        if constexpr (TCH > 0) asm volatile("s_waitcnt vmcnt(0)" : : "v"(touch_sink) : "memory");
        ++xi;
        clk.waited(a.stamps);
        ok = okf != 0;
        if (!ok || last) break;
        // h of block bd (MGS in exact arithmetic), the H column, the new Gram terms
        if (t == 0) {
            double hn[S];
#pragma unroll
            for (int k = 0; k < S; ++k)
                if (k < rd) {
                    double hk = bc[k];
#pragma unroll
                    for (int l = 0; l < k; ++l) {
                        const double g = (gram && k == rd - 1) ? bc[rd + l] : gbuf[(k - 1) * RES_SMAX + (k - l)];
                        hk = hk - hn[l] * g;
                    }
                    hn[k] = hk;
                }
#pragma unroll
            for (int s = 0; s < S; ++s) {  // slot s holds real column k = s - (S - rd)
                double v = 0.0;
#pragma unroll
                for (int k = 0; k < S; ++k)
                    if (k < rd && s == S - rd + k) v = hn[k];
                hv[s] = v;
            }
            if (blockIdx.x == 0) {
                const bool sw1 = p + 1 < nb1;  // block bd is subtracted in the first sweep
#pragma unroll
                for (int k = 0; k < S; ++k)
                    if (k < rd) hsh[id + k] = (sw1 ? 0.0 : hsh[id + k]) + hn[k];
                if (gram && sw1)
                    for (int l = 0; l < rd - 1; ++l) a.gm[(i64)(j - 1) * RES_SMAX + (rd - 1 - l)] = bc[rd + l];
            }
        }
        __syncthreads();
    }
    if (!ok) return;  // uniform per workgroup; *err is set
    const double hn = sqrt(bc[0]);
    double2 *__restrict__ O2 = reinterpret_cast<double2 *>(a.vout);
    auto outv = [&](const double2 &v) { return hn != 0.0 ? double2{v.x / hn, v.y / hn} : double2{0.0, 0.0}; };
    {
        int cb, ce;
        range(cb, ce);
#pragma unroll
        for (int k = 0; k < RW; ++k)
            if (cb + k < ce) O2[(i64)(cb + k) * NT + t] = outv(wr[k]);
    }
    for (int k = 0; k < LW; ++k)
        if (l0 + k < lend) O2[(l0 + k) * NT + t] = outv(lw[k * NT + t]);
    for (i64 e = a.nres2 + (i64)res_stream_wg() * NT + t; e < n2; e += sstride) O2[e] = outv(W2[e]);
    if ((a.n & 1) && blockIdx.x == gridDim.x - 1 && t == 0) a.vout[a.n - 1] = hn != 0.0 ? a.w[a.n - 1] / hn : 0.0;
    clk.finish(a.stamps, RES_MGS);
    if (blockIdx.x == 0) {
        __syncthreads();
        for (int k = t; k < j; k += NT) {
            a.hs[k] = hsh[k];
            a.hcopy[k] = hsh[k];
        }
        if (t == 0) {
            a.hs[j] = hn;
            a.hcopy[j] = hn;
        }
    }
}

// ------------------------------------------------------------------ host ---
#ifndef GK_BLK_KERNEL_ONLY  // (register-budget experiments instantiate one kernel themselves)
#ifndef GK_BLK_TOUCH
#define GK_BLK_TOUCH 28
#endif
constexpr int BLK_TOUCH = GK_BLK_TOUCH;  // the w-only build's touched chunks (k_mgs_wres's TOUCH_MGS)

namespace {

// register budget per S: two-wave builds hold 256 VGPRs per lane, the one-wave
// w-only build ~500; a larger S takes a shallower batch (the same loads in flight)
template <int S>
struct BlkCfg;
// (measured in the compile: the largest spill-free geometry of each variant; a
// deeper batch or more cached register chunks spilled)
// The LDS prefetch of the next dot block is capped at GK_BLK_PFX_KB per workgroup: about what
// HBM delivers to one CU during an all-gather -- the rest streams in the pass, where compute
// overlaps it, instead of holding the pass back at the wait for the prefetch (96 vs 128 / 80:
// 1024^2 S = 4 2.44 -> 2.30 us per projection, 1448^2 S = 2 4.25 -> 4.07, S = 4 3.95 -> 3.90;
// profiles/r05/ab_blk_pfx_kb_r05ae.txt)
#ifndef GK_BLK_PFX_KB
#define GK_BLK_PFX_KB 96
#endif
constexpr int pfx_cap(int chunks, int S, int nt) {
    const int c = GK_BLK_PFX_KB * 1024 / (S * nt * 16);
    return chunks < c ? chunks : c;
}
#ifndef GK_BLK_S1_R32_RX
#define GK_BLK_S1_R32_RX 8
#endif
// S = 1: the strict MGS-R step (h = <w, V_k> after the AXPY of V_{k-1}: gmres_mgsr.f90:341-360 in
// its order) on this kernel's LDS prefetch of the next dot column during the all-gather
// (GK_TUNE_RES_PF): the whole column for <= 16 chunks, RX of 32 otherwise (16 spilled)
template <>
struct BlkCfg<1> {
    static constexpr BlkGeom g[BLK_NVAR] = {{4, 0, 4, 0, 512, pfx_cap(4, 1, 512)},
                                            {8, 0, 8, 0, 512, pfx_cap(8, 1, 512)},
                                            {16, 0, 16, 0, 512, pfx_cap(16, 1, 512)},
                                            {32, 0, GK_BLK_S1_R32_RX, 0, 512, pfx_cap(GK_BLK_S1_R32_RX, 1, 512)},
                                            {90, 38, 0, 0, 256, 0}};
    static constexpr int wb[BLK_NVAR] = {4, 4, 4, 2, 4};
};
// (S = 2 at 16 chunks as a one-wave build -- the whole slab and both columns in registers, half
// the next dot block prefetched -- was slower: 2048^2 8.04 -> 8.84 us per projection, its
// all-gather wait 2.1 -> 3.2 us; profiles/r05/ab_blk_s2_onewave_r05v.txt)
template <>
struct BlkCfg<2> {
    static constexpr BlkGeom g[BLK_NVAR] = {{4, 0, 4, 0, 512, pfx_cap(4, 2, 512)},
                                            {8, 0, 8, 0, 512, pfx_cap(8, 2, 512)}, {16, 0, 7, 9, 512, 0},
                                            {32, 0, 1, 9, 512, 0}, {90, 38, 0, 0, 256, 0}};
    static constexpr int wb[BLK_NVAR] = {4, 4, 4, 2, 4};
};
#ifndef GK_BLK_S4_R8_1W
#define GK_BLK_S4_R8_1W 1
#endif
// S = 4 at <= 8 chunks of 512 (the 4096^2 / 8 load): one wave per SIMD -- 16 chunks of w and
// of each of the 4 cached columns in ~450 registers -- so that LDS is free for the first 8
// chunks of the next dot block, prefetched during the all-gather (the two-wave build had no
// room for either prefetch or cache: 4.32 -> 4.12 us per projection at 1448^2,
// profiles/r05/ab_blk_s4_onewave_r05t.txt)
template <>
struct BlkCfg<4> {
    static constexpr BlkGeom g[BLK_NVAR] = {{4, 0, 4, 0, 512, pfx_cap(4, 4, 512)},
                                            GK_BLK_S4_R8_1W ? BlkGeom{16, 0, 16, 0, 256, pfx_cap(8, 4, 256)} : BlkGeom{8, 0, 8, 0, 512, 0},
                                            {16, 0, 2, 4, 512, 0}, {32, 0, 0, 4, 512, 0}, {88, 38, 0, 0, 256, 0}};
    static constexpr int wb[BLK_NVAR] = {4, GK_BLK_S4_R8_1W ? 4 : 2, 2, 1, 2};
};

template <int S, int V>
int launch_v(const ResArgs &a, int G, int lds, int dev, hipStream_t st) {
    constexpr BlkGeom g = BlkCfg<S>::g[V];
    constexpr int WBT = BlkCfg<S>::wb[V];
    constexpr int TCH = V == BLK_WONLY ? BLK_TOUCH : 0;
    auto kern = &k_mgs_blk<g.rw, g.lw, g.rx, g.lx, S, WBT, TCH, g.nt, g.pfx>;
    static std::atomic<int> attr[64];
    if (dev < 0 || dev >= 64) return (int)hipErrorInvalidDevice;
    if (lds > 0 && attr[dev].load() < lds) {
        const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(kern),
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, lds);
        if (e != hipSuccess) return (int)e;
        attr[dev] = lds;
    }
    kern<<<G, g.nt, lds, st>>>(a);
    return (int)hipGetLastError();
}

template <int S>
int launch_s(int var, const ResArgs &a, int G, int lds, int dev, hipStream_t st) {
    switch (var) {
        case BLK_R4: return launch_v<S, BLK_R4>(a, G, lds, dev, st);
        case BLK_R8: return launch_v<S, BLK_R8>(a, G, lds, dev, st);
        case BLK_R16: return launch_v<S, BLK_R16>(a, G, lds, dev, st);
        case BLK_R32: return launch_v<S, BLK_R32>(a, G, lds, dev, st);
        case BLK_WONLY: return launch_v<S, BLK_WONLY>(a, G, lds, dev, st);
        default: return (int)hipErrorInvalidValue;
    }
}

}  // namespace

BlkGeom blk_geom(int var, int S) {
    if (var < 0 || var >= BLK_NVAR) return BlkGeom{0, 0, 0, 0, 0, 0};
    return S == 4 ? BlkCfg<4>::g[var] : (S == 1 ? BlkCfg<1>::g[var] : BlkCfg<2>::g[var]);
}

int blk_variant(long long chunks512) {
    return chunks512 <= 4 ? BLK_R4 : chunks512 <= 8 ? BLK_R8 : chunks512 <= 16 ? BLK_R16 : chunks512 <= 32 ? BLK_R32 : BLK_WONLY;
}

int blk_launch(int var, int S, const ResArgs &a, int G, int lds, int dev, hipStream_t st) {
    switch (S) {
        case 1: return var == BLK_WONLY ? (int)hipErrorInvalidValue : launch_s<1>(var, a, G, lds, dev, st);
        case 2: return launch_s<2>(var, a, G, lds, dev, st);
        case 4: return launch_s<4>(var, a, G, lds, dev, st);
        default: return (int)hipErrorInvalidValue;
    }
}

#endif  // GK_BLK_KERNEL_ONLY

}  // namespace gk
