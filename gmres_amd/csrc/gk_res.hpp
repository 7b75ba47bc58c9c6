// gk_res.hpp -- device-side machinery shared by the resident MGS-R / Householder
// step kernels (gk_kernels.hpp, gk_blk.hip): the device-exchange granule
// primitives, ResArgs and the in-launch all-gather.  Only inline functions,
// constants and types: included by more than one translation unit.
#pragma once
#include "gk_common.hpp"
#include "gk_cheb.hpp"

namespace gk {

// --------------------------------------------------------------------------
// Device-initiated exchange between ranks (the "xgmi" collective back-end).
//
// Every rank owns one receive region in uncached HBM that is mapped into every
// peer (IPC handles across processes, plain pointers inside one process).  A
// value travels as granules: one 8-byte word {32 data bits | 32-bit tag}
// written by ONE system-scope 8-byte store, so a receiver that reads the tag of
// the current exchange also reads its data -- no separate flag, no fence.
// Slots are double-buffered by the parity of the exchange sequence number.
// Every exchange is a rendezvous (each rank waits for the granules of every
// rank it receives from), so no rank gets two exchanges ahead of a partner and
// a slot is never overwritten before it has been read.  Every wait is bounded
// by a wall-clock deadline: a missing peer sets the context's error flag
// instead of hanging the GPU, and every later exchange returns NaN at once.
//
// Region layout (8-byte words):
//   reductions  [parity 2][source rank XS_MAXR][value XS_MAXV][half 2]
//   halo lines  [parity 2][side 2][N][half 2]   side 0: from rank-1, 1: from rank+1
// --------------------------------------------------------------------------
constexpr int XS_MAXR = 16;
constexpr int XS_MAXV = 128;
constexpr i64 XS_RED_WORDS = 2LL * XS_MAXR * XS_MAXV * 2;
typedef unsigned long long u64;
struct XsPeers {
    u64 *p[XS_MAXR];
};
enum { XS_SLAB = 0, XS_VEC = 1, XS_BCAST = 2 };

__device__ __forceinline__ void xs_put(u64 *q, unsigned seq, unsigned data) {
    __hip_atomic_store(q, ((u64)seq << 32) | data, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ int xs_flag(const int *err) {
    return __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Spin until the granule at q carries `seq`: XG_OK; XG_LATE once the deadline
// passed (the caller names the straggler); XG_ABORT when another wait of this
// rank already failed (the sticky flag *err is set, checked every 32 unanswered
// polls): the exchange is dead, so a doomed launch ends within microseconds
// instead of waiting out its own deadline, and the first failure stays the one
// reported.
enum { XG_ABORT = -1, XG_LATE = 0, XG_OK = 1 };
__device__ __forceinline__ int xs_get(const u64 *q, unsigned seq, u64 deadline, unsigned *data, const int *err) {
    for (unsigned it = 1;; ++it) {
        const u64 g = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if ((unsigned)(g >> 32) == seq) {
            *data = (unsigned)g;
            return XG_OK;
        }
        if (wall_clock64() > deadline) return XG_LATE;
        if ((it & 31u) == 0 && xs_flag(err) != 0) return XG_ABORT;
        __builtin_amdgcn_s_sleep(2);
    }
}

// Which wait missed its deadline (straggler diagnostic, decoded by the host
// into gk_last_error): code = op << 16 | (source + 1); source = the rank (or,
// for XSE_RES_WG, the workgroup of this rank) whose granule never came.  A
// plain store into mapped host memory (no read-modify-write over PCIe): with
// several failing waits the last one is reported.
enum { XSE_XCHG = 1, XSE_BCAST = 2, XSE_HALO = 3, XSE_RES_WG = 4, XSE_RES_RANK = 5 };
__device__ __forceinline__ void xs_fail(int *err, int op, int src) {
    __hip_atomic_store(err, (op << 16) | ((src + 1) & 0xFFFF), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// --------------------------------------------------------------------------
// Resident MGS-R step (gmres_mgsr.f90:341-363, :384): ONE persistent launch
// runs the whole cascade of Arnoldi step j -- 2j projections, the norm and
// V(:,j+1) = w/h -- instead of 2j+1 launches.  The first `nres2` double2 of w,
// and of the Krylov column the running projection needs, stay in registers
// for the whole step, so that part of the vector moves 8 B/unknown per
// projection (the next column) instead of k_proj's 32; the rest of the vector
// streams exactly as in k_proj.  With PF the next column is loaded before the
// wait for the current dot (its loads overlap the all-gather).
//
// The dot of each projection is all-gathered inside the launch: every
// workgroup publishes its partial as two tagged 8-byte granules (the data is
// the flag: cdna_hip_programming.md Guideline 16 R2 -- no fence, no counter),
// one wave of every workgroup sweeps all G partials (8 granules in flight per
// lane) and sums them in a fixed order, so every workgroup computes the
// bit-identical h and the launch is deterministic.  On N ranks the rank
// totals then travel through the device exchange regions (k_xchg's slots and
// sequence numbers) and are summed in rank order.  Every wait is bounded by a
// wall-clock deadline; a miss sets *err and ends the launch (results
// poisoned, the host reports the error).  The grid must be co-resident: one
// workgroup per CU, pinned there by its dynamic LDS.
// Element-wise arithmetic is k_proj's / k_scale's (bit-identical); only the
// dot summation order differs.
// --------------------------------------------------------------------------
constexpr int RT = 512;       // threads per resident workgroup (8 waves, 2 per SIMD)
constexpr int RWAVES = RT / 64;
constexpr int RGMAX = 1024;   // max workgroups of a resident launch
constexpr int RHMAX = 512;    // max m on the resident path (H column in LDS)
constexpr int WO_HMAX = 500;  // ... on the w-only MGS step (its LDS holds 39 chunks of w: k_mgs_wres)

struct ResArgs {
    double *w;            // w = M^-1 A V(:,j) from the operator launch; streamed part in/out
    const double *V;      // Krylov basis, column stride ld (doubles, even)
    double *vout;         // V(:,j+1)
    i64 ld;
    const double *pin;    // partial slab of <w, V(:,1)> (operator launch; all-reduced on N ranks)
    int npin;
    double *hs;           // H(1:j+1, j) on device
    double *hcopy;        // mapped host mirror of H(1:j+1, j)
    u64 *gath;            // [2][gridDim.x][2] granules
    int *err;             // mapped error flag
    u64 timeout;          // wall-clock ticks per wait
    unsigned tag0;        // granule tag of exchange p = tag0 + p (never 0)
    int j;
    i64 n, nres2;         // local length; resident double2 prefix
    i64 unit_e;           // RES_HH_DOWN with unit_known: local index of the input's 1.0 (-1: other rank)
    int unit_known;       // the input vector is a unit vector: leading dot = one element, no pass
    int r2e, l2e;         // chunks per workgroup actually resident in registers / LDS (<= the
                          // template's R2 / L2): the resident prefix is spread evenly
    XsPeers peers;        // nranks > 1: device exchange regions
    int nranks, rank;
    unsigned xseq0;       // exchange p uses sequence number xseq0 + 1 + p
    int mode;             // RES_MGS / RES_HH_UP / RES_HH_DOWN (res_col)
    double coef;          // AXPY coefficient: w -= (coef*h) V_i (1 for MGS, 2 for reflections)
    i64 tail0;            // RES_HH_UP: the closing norm counts local indices >= tail0
    u64 *stamps;          // profiling (nullptr = off): [mode][workgroup][pass, wait, total, launches] ticks
    // w-only kernel (k_mgs_wres) only:
    int close_hh;         // RES_HH_UP: the launch also makes the next reflector (gmres_hh.f90:306-318):
                          // w(1:j) = 0, w(j+1) += sign, P(:,j+1) = w / ||w|| to vout (w not written back)
    double *hb;           // close_hh: w(1:j+1) before the fix-up, written by the owner rank (pivot input)
    int unit_init;        // RES_HH_DOWN with unit_known: the launch builds e_u itself (w not read)
    u64 *trace;           // gk_profile_res_trace (nullptr = off): [workgroup][RES_TRACE_X][publish, seen] ticks
    // k_mgs_res with NT: the LDS-held and streamed parts load their dot column V_q
    // with the default policy (it is the next pass's AXPY column V_i: then an
    // Infinity-Cache hit), V_i non-temporal -- the w-only kernel's policy
    int qdef;
    int pin_local;        // N ranks, MGS: pin is this rank's partial slab only (res_pin_fold)
    // blocked step (k_mgs_blk) only: the Gram table of the cycle's basis, gm[c * RES_SMAX + d] =
    // <V(:,c-d+1), V(:,c+1)> for the columns c-d, c (0-based) of one projection block
    double *gm;
};
constexpr int RES_TRACE_X = 2 * RHMAX + 2;  // exchanges recorded per workgroup (all of one launch)

// Time split of a resident launch (gk_profile_res_split): thread 0 of each
// workgroup accumulates wall-clock ticks spent streaming its passes and waiting
// in the all-gathers into its own slot (no contention, plain adds).
struct ResClock {
    u64 t0 = 0, tp = 0, pass = 0, wait = 0;
    __device__ __forceinline__ void start(const u64 *st) {
        if (st != nullptr) t0 = tp = wall_clock64();
    }
    __device__ __forceinline__ void passed(const u64 *st) {  // a pass ended, its exchange starts
        if (st != nullptr) {
            const u64 n = wall_clock64();
            pass += n - tp;
            tp = n;
        }
    }
    __device__ __forceinline__ void waited(const u64 *st) {  // the exchange returned
        if (st != nullptr) {
            const u64 n = wall_clock64();
            wait += n - tp;
            tp = n;
        }
    }
    __device__ __forceinline__ void finish(u64 *st, int mode) {
        if (st != nullptr && threadIdx.x == 0) {
            u64 *q = st + 4 * ((i64)mode * RGMAX + blockIdx.x);
            q[0] += pass;
            q[1] += wait;
            q[2] += wall_clock64() - t0;
            q[3] += 1;
        }
    }
};

// Projection sequences of a resident launch (all columns of V, stride ld):
//  RES_MGS     gmres_mgsr.f90:341-363   2j projections i = p mod j, pre-dot from
//              pin, closes with ||w||, V(:,j+1) = w/||w|| and H(1:j+1,j)
//  RES_HH_UP   gmres_hh.f90:290-305     w = P_j..P_1 w: i = p (p < j), pre-dot
//              from pin, closes with ||w(j+1:n)||^2 -> hs[0]; w back to HBM
//  RES_HH_DOWN gmres_hh.f90:269-283     v = P_1..P_j v: i = j-1-p, the pre-dot
//              is computed in the launch, no closing reduction; v back to HBM
// A reflection is the projection with coef 2 (w -= 2<w,P_i> P_i).
enum { RES_MGS = 0, RES_HH_UP = 1, RES_HH_DOWN = 2 };
enum { RK_NONE = 0, RK_DOT = 1, RK_NORM = 2 };  // reduction closing a pass

// The streamed elements (past the resident chunks) go to the workgroups from the LAST one
// down: when the resident chunks do not fill the grid (1448^2, 2896^2: a ragged last chunk)
// the last workgroup's chunk range is the short one, so the ragged tail rides there instead
// of lengthening workgroup 0's pass -- which the all-gather trace showed as the straggler of
// every exchange (profiles/r05/res_trace_1448_r05ac.txt; A/B ab_stream_wg_r05ad.txt, _4096_r05ag.txt)
__device__ __forceinline__ unsigned res_stream_wg() { return gridDim.x - 1 - blockIdx.x; }

__device__ __forceinline__ int res_np(int mode, int j) { return mode == RES_MGS ? 2 * j : j; }
__device__ __forceinline__ int res_col(int mode, int j, int p) {
    const int np = res_np(mode, j);
    p = p < np ? p : np - 1;
    return mode == RES_MGS ? p % j : (mode == RES_HH_UP ? p : j - 1 - p);
}

// acc += v.x^2 + v.y^2 for the element pair of local double2 index e2; with chk
// only the elements at local index >= tail0.  tail0 <= j <= RHMAX lies inside the
// first chunk of the vector, so callers pass a uniform chk that is true for that
// chunk only (RES_HH_UP): the per-element test stays out of every other chunk,
// and out of the register allocation of the steady-state loop.
__device__ __forceinline__ void sq_acc(double &acc, const double2 &v, i64 e2, i64 tail0, bool chk) {
    if (chk) {
        if (2 * e2 >= tail0) acc = acc + v.x * v.x;
        if (2 * e2 + 1 >= tail0) acc = acc + v.y * v.y;
    } else {
        acc = acc + v.x * v.x;
        acc = acc + v.y * v.y;
    }
}

__device__ __forceinline__ double block_sum_rt(double v, double *sm) {
    v = wave_sum(v);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) sm[wid] = v;
    __syncthreads();
    double r = sm[0];
#pragma unroll
    for (int k = 1; k < RWAVES; ++k) r += sm[k];
    __syncthreads();  // sm is rewritten next
    return r;
}

// Wave 0 of every workgroup: sum the workgroup's wave partials sm[0..RWAVES)
// in order, publish that sum of exchange p as two tagged granules, sweep the
// G partials of the grid (8 granules in flight per lane) and sum them in a
// fixed order; on N ranks then add the rank totals in rank order.  Result in
// bc[0]; *okf = 0 when a deadline passed (then *err is set).
// (Round 5: the two-hop all-gather -- 8 group leaders summing their members and
// publishing group sums, GK_RES_XHOPS 2 -- was removed from the kernels.  It won at
// 1024^2 only while one granule array was swept by all 256 workgroups, 4.25 vs 4.37
// us per projection (profiles/r02/ab_hops_*.jsonl); with the replicas below the flat
// sweep is faster there too, 3.88 vs 4.1 us (profiles/r02/ab_nrep_1024.jsonl), and it
// always was at 2048^2 (10.4 vs 10.9) and 4096^2 (41.6 vs 43.2).)
#ifndef GK_RES_NREP
#define GK_RES_NREP 8
#endif
// Replicas of the granule array: every workgroup publishes its partial into all
// RES_NREP copies (one store per lane of 2 * NREP lanes) and sweeps copy
// blockIdx % NREP -- under round-robin dispatch the copy of its own XCD, never
// assumed for correctness -- so each copy's lines are polled by 1/NREP of the
// grid instead of all of it (MI355X_MICROARCH.md allgather: 256 -> 32 readers
// -1.9 us on a 16 KB sweep).  Copies RES_REP_STRIDE words apart (a 256 B skew on
// top of the array size, so they fall on different channels).  1 = one array.
constexpr int RES_NREP = GK_RES_NREP;
constexpr i64 RES_REP_STRIDE = 4 * (i64)RGMAX + 32;
constexpr i64 RES_REP0 = 4 * (i64)RGMAX + 32;  // first replica (RES_NREP > 1)
// [2][RGMAX][2] partials + 32 words (once the two-hop group sums) + the replicas
constexpr i64 RES_GATH_WORDS = RES_REP0 + (RES_NREP > 1 ? RES_NREP * RES_REP_STRIDE : 0);
// rank totals of the resident launches: replica r in value slot XS_REP_STEP * r (128 B apart)
constexpr int XS_REP_STEP = 8;
static_assert(RES_NREP >= 1 && RES_NREP * XS_REP_STEP <= XS_MAXV, "replicas must fit the exchange value slots");

#ifndef GK_RES_POLL_SLEEP
#define GK_RES_POLL_SLEEP 16
#endif
#ifndef GK_RES_POLL_SLEEP_SMALL
#define GK_RES_POLL_SLEEP_SMALL 4
#endif
// s_sleep units (64 clocks) between unanswered polls, per kernel: the w-only
// large-slab kernel (RES_POLL_SLEEP) and k_mgs_res (RES_POLL_SLEEP_SMALL).  A/B with
// one granule array (profiles/r02/ab_poll_*.jsonl): 1 / 4 / 16 / 48 -> 4096^2 42.1 / 42.1
// / 41.7 / 41.6 us, 1024^2 4.42 / 4.45 / 4.40 / 4.81 us per projection: continuous polls
// by early finishers slow the stragglers' streams.  With 8 replicas
// (profiles/r02/ab_rep_*.jsonl) 4 instead of 16: 4096^2 41.8 vs 41.5 us, but 2048^2 9.57
// vs 9.66 and 1024^2 4.12 vs 4.28 -- a poll is cheaper once 32 readers share a copy.
constexpr int RES_POLL_SLEEP = GK_RES_POLL_SLEEP;
#ifndef GK_RES_PUSHER_FAST
#define GK_RES_PUSHER_FAST 1
#endif
// N ranks: workgroup 0, which pushes the rank total to the peers once its sweep
// completes, polls its granules without the sleep (its detection delay is on
// every rank's critical path; the other workgroups' is not).
constexpr bool RES_PUSHER_FAST = GK_RES_PUSHER_FAST != 0;
#ifndef GK_RES_PUSHERS
#define GK_RES_PUSHERS 4
#endif
// N ranks: workgroups 0 .. RES_PUSHERS-1 (one per XCD under round-robin dispatch)
// each sweep this rank's granules and push the same rank total (same bits, same
// sequence tag) into every peer slot, so a total lands as soon as the FIRST of them
// has seen the sweep complete.  A pusher's stores are complete before it publishes
// its next partial (s_waitcnt below), so no push of exchange p can land on a slot
// after the same-parity push of exchange p + 2.  Same-device rehearsals, 1 / 4 / 8
// pushers, three alternating samples (profiles/r05/ab_pushers_r05j.jsonl; every run
// the same bits): wait per projection 2 ranks 2896^2 4.67 / 4.57 / 4.58 us (one
// outlier of 1 and 8 dropped), 4 ranks 2048^2 4.01 / 3.93 / 4.02, 2 ranks 1448^2
// 3.81 / 3.79 / 3.89 -- a small gain at 4, none at 8.
constexpr int RES_PUSHERS = GK_RES_PUSHERS;
static_assert(RES_PUSHERS >= 1 && RES_PUSHERS <= 8, "1..8 rank-total pushers");
__device__ __forceinline__ bool res_pusher(const ResArgs &a) { return a.nranks > 1 && blockIdx.x < RES_PUSHERS; }
// N ranks: only the pushers (workgroup 0 by default) sweep the local granules (every workgroup reads the R
// rank totals, its own rank's among them).  Round 5 removed the A/B knob that let
// every workgroup sweep (GK_RES_SWEEP_ALL): the same bits, a tie in the same-device
// rehearsals (profiles/r04/ab_sweep_r04x.jsonl: 605 / 601, 1,094 / 1,093, 1,546 /
// 1,529 it/s pusher-only / all).
constexpr int RES_POLL_SLEEP_SMALL = GK_RES_POLL_SLEEP_SMALL;
#ifndef GK_RES_POLL_SLEEP_PC
#define GK_RES_POLL_SLEEP_PC 16
#endif
// the column-cache kernel k_mgs_wpc (A/B knob)
constexpr int RES_POLL_SLEEP_PC = GK_RES_POLL_SLEEP_PC;

// Wave 0 of every workgroup, N ranks: the rank totals of exchange index p
// (sequence number a.xseq0 + 1 + p).
// v: value index of a multi-value exchange (the blocked step, k_mgs_blk): value slot
// XS_REP_STEP * r + v of each replica r.
__device__ __forceinline__ double res_rank_sum(const ResArgs &a, int p, double acc, bool &all_ok, int v = 0) {
    const int lane = threadIdx.x & 63;  // any one wave of the workgroup (value v on wave v in k_mgs_blk)
    // Rank totals: the pushers (workgroup 0 by default) push this rank's total into every peer's region,
    // once per replica (value slot XS_REP_STEP * r of its source row: a line of its
    // own), and every workgroup reads replica blockIdx % NREP -- 1/NREP of the grid
    // polls each line instead of all of it.  A slot is rewritten two exchanges later
    // at the earliest, after every workgroup of every rank has read it (rendezvous).
    const unsigned seq = a.xseq0 + 1u + (unsigned)p, par = seq & 1u;
    if (blockIdx.x < RES_PUSHERS) {
        const u64 bits = (u64)__double_as_longlong(acc);
        for (int k = lane; k < 2 * RES_NREP * a.nranks; k += 64) {
            const int dst = k / (2 * RES_NREP), r = (k >> 1) % RES_NREP, half = k & 1;
            xs_put(a.peers.p[dst] + (((i64)par * XS_MAXR + a.rank) * XS_MAXV + XS_REP_STEP * r + v) * 2 + half, seq,
                   half ? (unsigned)(bits >> 32) : (unsigned)bits);
        }
    }
    unsigned d = 0;
    bool ok2 = true;
    if (lane < 2 * a.nranks) {
        const int src = lane >> 1, half = lane & 1, r = (int)(blockIdx.x % RES_NREP);
        const int g = xs_get(a.peers.p[a.rank] + (((i64)par * XS_MAXR + src) * XS_MAXV + XS_REP_STEP * r + v) * 2 + half,
                             seq, wall_clock64() + a.timeout, &d, a.err);
        ok2 = g == XG_OK;
        if (g == XG_LATE) xs_fail(a.err, XSE_RES_RANK, src);
    }
    all_ok = all_ok && __all(ok2);
    double r = 0.0;
    for (int q = 0; q < a.nranks; ++q) {  // rank order, as k_xchg<XS_SLAB>
        const unsigned lo = __shfl(d, 2 * q, 64), hi = __shfl(d, 2 * q + 1, 64);
        const double v = __longlong_as_double((long long)(((u64)hi << 32) | lo));
        r = (q == 0) ? v : r + v;
    }
    return r;
}

// pin_local (N ranks, the MGS step): the stencil's first-dot partial slab `pin`
// is this rank's alone -- no k_xchg launch before the step -- and its total h
// goes through the rank-total hop here (exchange index -1, the launch's first
// sequence number), summed in rank order like every in-launch total.
__device__ __forceinline__ bool res_pin_fold(const ResArgs &a, double &h, double *bc, int *okf) {
    if (!a.pin_local) return true;
    if (threadIdx.x < 64) {
        bool ok = true;
        const double r = res_rank_sum(a, -1, h, ok);
        if (threadIdx.x == 0) {
            bc[0] = r;
            *okf = ok ? 1 : 0;
        }
    }
    __syncthreads();
    h = bc[0];
    return *okf != 0;
}

// TR: the trace stamps (gk_profile_res_trace) are compiled into the MGS-R launches only
// (the reflection kernels are at the edge of the register file).
template <int NW = RWAVES, bool TR = false, int SLEEP = RES_POLL_SLEEP>
__device__ __forceinline__ void res_exchange(const ResArgs &a, int p, const double *sm, double *bc, int *okf) {
    const int lane = threadIdx.x;
    const int G = gridDim.x;
    const unsigned tag = a.tag0 + (unsigned)p;
    auto rep_slot = [&](int r) -> u64 * {  // granule array of exchange p in replica r
        return a.gath + (RES_NREP > 1 ? RES_REP0 + r * RES_REP_STRIDE : 0) + (i64)(p & 1) * G * 2;
    };
    u64 *slot = rep_slot((int)(blockIdx.x % RES_NREP));  // the copy this workgroup sweeps
    double s = sm[0];
#pragma unroll
    for (int w = 1; w < NW; ++w) s += sm[w];
    u64 t_pub = 0;
    if (TR && a.trace != nullptr) t_pub = wall_clock64();
    if (RES_PUSHERS > 1 && res_pusher(a)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the last push landed
    if (lane < 2 * RES_NREP) {  // lane 2r + h: half h of the partial into replica r
        const u64 bits = (u64)__double_as_longlong(s);
        const int half = lane & 1;
        __hip_atomic_store(rep_slot(lane >> 1) + 2 * blockIdx.x + half,
                           ((u64)tag << 32) | (half ? (unsigned)(bits >> 32) : (unsigned)bits), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
    const u64 deadline = wall_clock64() + a.timeout;
    double acc = 0.0;
    bool all_ok = true;
    if (a.nranks == 1 || blockIdx.x < RES_PUSHERS) {
        // (N ranks: only the pushers need this rank's total -- every
        // workgroup then reads the R rank totals, its own rank's included, so the
        // others skip the sweep and its polls stay off the stragglers' memory path.)
        // Lane L holds granule L + 64k of each 512-granule sweep: the lo (even L)
        // or hi (odd L) half of workgroup c0/2 + L/2 + 32k.
        for (int c0 = 0; c0 < 2 * G && all_ok; c0 += 512) {
            unsigned v[8];
            for (;;) {
                // All 8 loads unconditionally (out-of-range lanes re-read granule 0
                // and ignore it): a per-load bounds branch made the compiler wait for
                // each load before issuing the next -- 8 serial round trips to the
                // point of coherence per poll instead of one.
                u64 x[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    const int g = c0 + lane + 64 * k;
                    x[k] = __hip_atomic_load(slot + (g < 2 * G ? g : 0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                bool ok = true;
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    const bool in = c0 + lane + 64 * k < 2 * G;
                    v[k] = in ? (unsigned)x[k] : 0u;
                    ok = ok && (!in || (unsigned)(x[k] >> 32) == tag);
                }
                if (__all(ok)) break;
                if (wall_clock64() > deadline) {
                    all_ok = false;
                    int miss = 0x7FFF;  // the lowest workgroup whose granule never came
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        const int g = c0 + lane + 64 * k;
                        if (g < 2 * G && (unsigned)(__hip_atomic_load(slot + g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                                    >> 32) != tag)
                            miss = min(miss, g >> 1);
                    }
                    for (int o = 32; o > 0; o >>= 1) miss = min(miss, __shfl_xor(miss, o, 64));
                    if (lane == 0) xs_fail(a.err, XSE_RES_WG, miss);
                    break;
                }
                if (RES_PUSHER_FAST && res_pusher(a))
                    __builtin_amdgcn_s_sleep(1);  // the rank-total pusher: push as soon as the sweep completes
                else
                    __builtin_amdgcn_s_sleep(SLEEP);
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) {  // workgroups in increasing order per lane pair
                const unsigned o = __shfl_xor(v[k], 1, 64);
                const unsigned lo = (lane & 1) ? o : v[k], hi = (lane & 1) ? v[k] : o;
                if (!(lane & 1) && c0 + lane + 64 * k < 2 * G)
                    acc = acc + __longlong_as_double((long long)(((u64)hi << 32) | lo));
            }
        }
        acc = wave_sum(acc);  // butterfly: the same value on every lane of every workgroup
    }
    if (all_ok && a.nranks > 1) acc = res_rank_sum(a, p, acc, all_ok);
    if (lane == 0) {
        bc[0] = acc;
        *okf = all_ok ? 1 : 0;
        if (TR && a.trace != nullptr && p < RES_TRACE_X) {
            u64 *q = a.trace + ((i64)blockIdx.x * RES_TRACE_X + p) * 2;
            q[0] = t_pub;
            q[1] = wall_clock64();
        }
    }
}

// --------------------------------------------------------------------------
// Multi-value all-gather of the blocked-projection step (k_mgs_blk, gk_blk.hip):
// one exchange carries K <= RES_KMAX values per workgroup -- the dots of a block
// of projections and the block's new Gram terms.  Value v has a granule array
// of its own (the single-value layout, RES_GATH_WORDS words, at v * RES_GATH_WORDS)
// and is all-gathered by wave v % NW of every workgroup with res_exchange's flat
// sweep and rank-total hop (value slot v of each replica), so K values cost the
// latency of one exchange, not K.
// --------------------------------------------------------------------------
constexpr int RES_SMAX = 4;                    // largest block of projections
constexpr int RES_KMAX = 2 * RES_SMAX - 1;     // its dots + the Gram terms of its newest column
constexpr i64 RES_GATH_ALL = (i64)RES_KMAX * RES_GATH_WORDS;
static_assert(RES_KMAX <= XS_REP_STEP, "the values of one exchange must fit a replica's value slots");

// One wave: publish value v of exchange p (s = this workgroup's partial of it) --
// its granule pair into every replica, no wait.
__device__ __forceinline__ void res_publish_v(const ResArgs &a, int p, int v, double s) {
    const int lane = threadIdx.x & 63;
    const unsigned tag = a.tag0 + (unsigned)p;
    if (lane < 2 * RES_NREP) {
        u64 *gv = a.gath + (i64)v * RES_GATH_WORDS;
        u64 *q = gv + (RES_NREP > 1 ? RES_REP0 + (lane >> 1) * RES_REP_STRIDE : 0) + (i64)(p & 1) * gridDim.x * 2;
        const u64 bits = (u64)__double_as_longlong(s);
        const int half = lane & 1;
        __hip_atomic_store(q + 2 * blockIdx.x + half, ((u64)tag << 32) | (half ? (unsigned)(bits >> 32) : (unsigned)bits),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// One wave: collect value v of exchange p -- sweep the G partials of this rank's
// copy (replica blockIdx % NREP; on N ranks the pushers only, then the rank-total
// hop).  Returns false when a deadline passed (*a.err set); *out = the grid (and
// rank) total, the same bits in every workgroup and on every rank.
template <int SLEEP>
__device__ __forceinline__ bool res_collect_v(const ResArgs &a, int p, int v, double *out) {
    const int lane = threadIdx.x & 63;
    const int G = gridDim.x;
    const unsigned tag = a.tag0 + (unsigned)p;
    const u64 *slot = a.gath + (i64)v * RES_GATH_WORDS +
                      (RES_NREP > 1 ? RES_REP0 + (int)(blockIdx.x % RES_NREP) * RES_REP_STRIDE : 0) + (i64)(p & 1) * G * 2;
    const u64 deadline = wall_clock64() + a.timeout;
    double acc = 0.0;
    bool all_ok = true;
    if (a.nranks == 1 || blockIdx.x < RES_PUSHERS) {  // (k_mgs_blk: every wave's stores drain before the
                                                     // barrier that ends an exchange, ahead of the next publish)
        for (int c0 = 0; c0 < 2 * G && all_ok; c0 += 512) {
            unsigned d[8];
            for (;;) {
                u64 x[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    const int g = c0 + lane + 64 * k;
                    x[k] = __hip_atomic_load(slot + (g < 2 * G ? g : 0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                bool ok = true;
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    const bool in = c0 + lane + 64 * k < 2 * G;
                    d[k] = in ? (unsigned)x[k] : 0u;
                    ok = ok && (!in || (unsigned)(x[k] >> 32) == tag);
                }
                if (__all(ok)) break;
                if (wall_clock64() > deadline) {
                    all_ok = false;
                    int miss = 0x7FFF;
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        const int g = c0 + lane + 64 * k;
                        if (g < 2 * G && (unsigned)(x[k] >> 32) != tag) miss = min(miss, g >> 1);
                    }
                    for (int o = 32; o > 0; o >>= 1) miss = min(miss, __shfl_xor(miss, o, 64));
                    if (lane == 0) xs_fail(a.err, XSE_RES_WG, miss);
                    break;
                }
                if (RES_PUSHER_FAST && a.nranks > 1)
                    __builtin_amdgcn_s_sleep(1);  // a rank-total pusher
                else
                    __builtin_amdgcn_s_sleep(SLEEP);
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) {  // workgroups in increasing order per lane pair
                const unsigned o = __shfl_xor(d[k], 1, 64);
                const unsigned lo = (lane & 1) ? o : d[k], hi = (lane & 1) ? d[k] : o;
                if (!(lane & 1) && c0 + lane + 64 * k < 2 * G)
                    acc = acc + __longlong_as_double((long long)(((u64)hi << 32) | lo));
            }
        }
        acc = wave_sum(acc);
    }
    if (all_ok && a.nranks > 1) acc = res_rank_sum(a, p, acc, all_ok, v);
    *out = acc;
    return all_ok;
}

}  // namespace gk
