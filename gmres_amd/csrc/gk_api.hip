// gk_api.hip -- C-ABI implementation of include/gmres_hip.h (libgmres_hip.so).
//
// One context per GPU (one process per GPU on a node).  A context owns the
// slab of grid lines [line0, line0+nlines) of every vector, the Krylov basis
// V (n_loc x (m+1), column stride padded to 256 B) and the reduction slabs,
// all resident in HBM for the whole solve; the host sees only the (j+1)
// Hessenberg entries of each Arnoldi step.  All work is issued on one HIP
// stream per context; on N GPUs the dot-product slabs are RCCL all-reduced
// and the stencil halos exchanged point-to-point on that same stream.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdarg>
#include <cstdlib>
#include <mutex>
#include <cstdio>
#include <cstring>
#include <deque>
#include <string>
#include <vector>

#include "../../include/gmres_hip.h"
#include "gk_blk.hpp"
#include "gk_kernels.hpp"
#include "gk_sr.hpp"

using gk::i64;

namespace {

thread_local std::string g_err;

int set_err(int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIPCHK(call)                                                                            \
    do {                                                                                        \
        hipError_t e_ = (call);                                                                 \
        if (e_ != hipSuccess) return set_err(GK_ERR_HIP, "%s:%d %s: %s", __FILE__, __LINE__, #call, \
                                             hipGetErrorString(e_));                            \
    } while (0)
#define NCCLCHK(call)                                                                           \
    do {                                                                                        \
        ncclResult_t r_ = (call);                                                               \
        if (r_ != ncclSuccess) return set_err(GK_ERR_RCCL, "%s:%d %s: %s", __FILE__, __LINE__, #call, \
                                              ncclGetErrorString(r_));                          \
    } while (0)
#define CHK(call)                      \
    do {                               \
        int s_ = (call);               \
        if (s_ != GK_OK) return s_;    \
    } while (0)
#define LAUNCHCHK() HIPCHK(hipGetLastError())

constexpr int NSLOT = 4;  // partial slabs (ping-pong + spares)
constexpr int PROF_POOL = 8192;

i64 round_up(i64 a, i64 b) { return (a + b - 1) / b * b; }

}  // namespace

// In-process communicator: several contexts of one process (e.g. ranks
// sharing one GPU in tests) driven by one host thread each.  Collectives are
// a host barrier + HIP event ordering + device copies/sums; the message
// pattern is exactly the RCCL one (same counts, same roots, same halos).
struct gk_group {
    int n = 0;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    long gen = 0;
    bool broken = false;
    std::vector<gk_ctx *> members;
    std::vector<const double *> ptrs;
};

struct gk_ctx {
    int dev = 0, N = 0, line0 = 0, nlines = 0, m = 0;
    i64 nloc = 0, ld = 0, g0 = 0;
    hipStream_t st = nullptr;
    // HBM residents
    double *V = nullptr;  // (m+1) columns, stride ld
    double *w = nullptr, *z = nullptr, *aux = nullptr, *dA = nullptr, *dB = nullptr;
    double *x = nullptr, *b = nullptr, *vj = nullptr, *hlo = nullptr, *hhi = nullptr;
    double *dh = nullptr;  // deep halos of the Chebyshev pass inputs: [3 vectors][lo, hi][CF_HMAX lines][N]
    double *zline = nullptr;  // N zeros (the short-recurrence marches' line past a physical boundary)
    double *red = nullptr;   // NSLOT * NPMAX partial slabs
    double *hcol = nullptr;  // m+2 Hessenberg column / scalars
    double *ydev = nullptr;  // m+1
    double *hb = nullptr;    // m+2 Householder broadcast buffer
    double *scal = nullptr;  // 8 scalars
    double *hcol_host = nullptr;  // pinned
    double *hall = nullptr;       // device: per-step Hessenberg columns, m slots of m+2
    double *hallh = nullptr;      // mapped pinned host mirror of hall (written by k_scale)
    double *hallh_dev = nullptr;  // its device address
    std::vector<hipEvent_t> ev_step;  // completion of step j
    double *Vb = nullptr;    // Householder verr basis (lazy)
    double *gram_slab = nullptr, *gram_out = nullptr;
    short2 *gram_pairs = nullptr;
    int gram_nblk = 0;
    // preconditioner
    int pkind = GK_PREC_IDENTITY, pdeg = 8;
    double p0 = 8.2, p1 = 0.2;
    // decomposition / comm
    int nranks = 1, rank = 0, max_lines = 0;
    int min_lines = 0;  // smallest slab of any rank (0: not gathered yet; ensure_min_lines)
    ncclComm_t comm = nullptr;
    bool comm_ok = false;
    gk_group *lg = nullptr;  // in-process group (GK local comm), else RCCL
    hipEvent_t lev_a = nullptr, lev_b = nullptr;
    double *lscratch = nullptr;
    // device exchange (xgmi back-end, gk_comm_init_xgmi / gk_xchg_*)
    gk::u64 *xs_buf = nullptr;  // own receive region, uncached HBM
    i64 xs_words = 0;
    gk::XsPeers xs_peers{};     // every rank's region, mapped here
    std::vector<void *> xs_mapped;
    bool xs_ready = false, xs_on = false, xs_broken = false;
    unsigned xs_seq = 0, xs_hseq = 0;
    int *xs_err = nullptr, *xs_err_dev = nullptr;  // mapped pinned flag
    long long xs_tick_per_ms = 100000;
    int xs_timeout_ms = 20000;
    gk::u64 xs_timeout = 0;
    // resident MGS-R step (gk::k_mgs_res): one persistent launch per Arnoldi step
    gk::u64 *res_gath = nullptr;                    // [RES_KMAX values][2][RGMAX][2] all-gather granules
    double *res_gm = nullptr;                       // blocked step: the cycle's Gram table [m+1][RES_SMAX]
    int tune_res_blk = 1;                           // blocked-projection MGS step: S (1 = strict MGS-R)
    int tune_res_pf = 0;                            // strict MGS step on the blocked kernel's LDS prefetch (S = 1)
    int pend_res_blk = 0, pend_res_pf = -1;         // requested mid-cycle: applied at the next cycle start
    int watchdog_ms = 0;                            // host watchdog of stream waits (0: from the device deadlines)
    bool broken = false;                            // the watchdog fired: a kernel of this context never completed
    unsigned *hold_word = nullptr, *hold_word_dev = nullptr;  // gk_debug_hold_stream's mapped word
    int *res_err = nullptr, *res_err_dev = nullptr;  // mapped deadline flag
    unsigned res_tag = 1;                           // next granule tag (never 0)
    int res_cus = 0;                                // compute units of the device
    int tune_res = -1;                              // -1 auto, 0 off, 1 on where possible
    int tune_res_r2 = 0;                            // cap of resident double2 per thread (0 = auto)
    int tune_res_lds = 1;                           // LDS-resident part of w for large slabs
    int tune_res_wonly = -1;                        // large slabs: w-only variant (-1: by the byte model)
    int tune_verr_order = 1;                        // v_err diagnostics in the reference's dot order
    int tune_hh_fuse = 1;                           // Householder step: small launches folded into the chains
    int tune_hh_norm_order = 0;                     // Householder: the reflector norms in flang-rt's order (1 rank)
    int res_share = 1;                              // contexts sharing this device's CUs
    int res_timeout_ms = 20000;
    bool res_broken = false;                        // a deadline was missed: launch path from then on
    gk::u64 *res_stamps = nullptr;                  // gk_profile_res_split: [RGMAX][4] ticks per workgroup
    bool res_split = false;
    gk::u64 *res_trace = nullptr;                   // gk_profile_res_trace: [RGMAX][RES_TRACE_X][2] ticks
    int res_trace_j = 0, res_trace_mode = -1;       // the traced launch: step j, mode (-1 = off)
    int res_trace_g = 0, res_trace_np = 0;          // its workgroups and exchanges
    // launch geometry
    int vec = 2, JT = 16;
    dim3 sgrid;
    int sr_JT = 64, tune_sr_blocks = 0;  // the short-recurrence marches' geometry (gk_sr_*)
    int tune_sr_two = 1;                 // GK_TUNE_SR_TWO_LEVEL
    bool sr_two = false;                 // this solve runs the two-level marches (set by gk_sr_start)
    dim3 sr_sgrid;
    int np_sr = 0;
    int np_st = 0, np_pj = 0, nblk_stream = 0;
    int last_np = 0;          // partial count written by the last ACC-carrying sweep
    int tune_cheb_fused = 1;  // temporal-blocked Chebyshev sweeps (single slab)
    int tune_cheb_sten = 1;   // the Arnoldi step's pass forms z = A v itself (stage 0)
    int tune_spin_wait = 1;   // the per-step host wait spins on its event (0: hipEventSynchronize)
    int tune_graph = 1;       // launch-path MGS-R steps captured as hipGraphs (RCCL / no collective)
    int tune_res_qdef = -1;   // k_mgs_res NT: V_q of the LDS / streamed parts with the default policy (-1 auto)
    int tune_res_pc = -1;     // column-cache variant k_mgs_wpc: -1 by the byte model, 0 never, 1 where it fits
    int tune_res_fold = 1;    // N ranks, device exchange: the first dot's rank hop inside the MGS step launch
    std::vector<hipGraphExec_t> gstep;  // captured step j (launch path), valid for partial-slab count gkey
    std::vector<unsigned> gxs;          // device exchanges in captured step j (their sequence numbers)
    int gkey = -1;
    unsigned graph_seq0 = 0;            // xs_seq when the capture in progress began
    unsigned *xs_seqdev = nullptr;      // device: the sequence base of a replayed graph's exchanges
    bool capturing = false;   // a step is being captured: no profiling events inside it
    // tuning knobs (gk_set_tuning)
    int tune_nt = -1, tune_pj_blocks = 0, tune_st_blocks = 0;  // tune_nt: -1 auto
    bool nt_auto = false;
    int tune_blocked = 0, tune_unr = 0;  // tune_unr 0 = auto
    int prof_every = 1;       // record events in steps with j % prof_every == 0
    bool prof_on_step = true;
    // state
    bool cycle_mgs = false, cycle_hh = false;
    double beta0 = -1.0;
    // profiling
    bool prof = false;
    std::vector<hipEvent_t> ev0, ev1;
    std::vector<int> evk;
    int nev = 0;
    double prof_ms[GK_NKID] = {0};
    long long prof_n[GK_NKID] = {0};
    // fused short-recurrence solve (gk_sr_*)
    gk::SrDev *sr_dev = nullptr;
    gk::SrMirror *sr_mir = nullptr, *sr_mir_dev = nullptr;  // mapped pinned
    double *sr_hist = nullptr;
    int sr_hist_len = 0;
    int sr_solver = -1, sr_par = 0, sr_queued = 0, sr_maxit = 0;
    std::deque<hipEvent_t> sr_pend;   // end of each queued chunk, oldest first
    std::vector<hipEvent_t> sr_evfree;
    hipGraphExec_t sr_graph = nullptr;  // SR_GRAPH_ITERS iterations from parity 0
};

namespace {

// ------------------------------------------------------------- profiling ---
int prof_harvest(gk_ctx *c) {
    if (c->nev == 0) return GK_OK;
    HIPCHK(hipEventSynchronize(c->ev1[c->nev - 1]));
    for (int k = 0; k < c->nev; ++k) {
        float ms = 0.f;
        HIPCHK(hipEventElapsedTime(&ms, c->ev0[k], c->ev1[k]));
        c->prof_ms[c->evk[k]] += ms;
        c->prof_n[c->evk[k]] += 1;
    }
    c->nev = 0;
    return GK_OK;
}

struct ProfScope {
    gk_ctx *c;
    int slot = -1;
    ProfScope(gk_ctx *c_, int kid) : c(c_) {
        if (!c->prof || !c->prof_on_step || c->capturing) return;
        if (c->nev == PROF_POOL) prof_harvest(c);
        slot = c->nev++;
        c->evk[slot] = kid;
        (void)hipEventRecord(c->ev0[slot], c->st);
    }
    ~ProfScope() {
        if (slot >= 0) (void)hipEventRecord(c->ev1[slot], c->st);
    }
};

double *slot(gk_ctx *c, int s) { return c->red + (i64)s * gk::NPMAX; }

// Captured launch-path steps hold kernel arguments and communicator calls of the
// configuration they were captured in: any change of tuning, preconditioner or
// communicator drops them.
void graph_reset(gk_ctx *c) {
    for (hipGraphExec_t &g : c->gstep)
        if (g != nullptr) {
            (void)hipGraphExecDestroy(g);
            g = nullptr;
        }
    c->gkey = -1;
    if (c->sr_graph != nullptr) {
        (void)hipGraphExecDestroy(c->sr_graph);
        c->sr_graph = nullptr;
    }
}

// ----------------------------------------------------------------- comm ---
constexpr int LG_MAX = 16;
struct RankPtrs {
    const double *p[LG_MAX];
};

__global__ void k_sum_ranks(RankPtrs src, int nr, double *__restrict__ out, int count) {
    for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < count; k += gridDim.x * blockDim.x) {
        double s = 0.0;
        for (int r = 0; r < nr; ++r) s += src.p[r][k];
        out[k] = s;
    }
}

// Collectives run whenever a communicator exists (also a 1-rank RCCL one).
bool collective(const gk_ctx *c) { return c->xs_on || c->comm != nullptr || c->lg != nullptr; }

// ------------------------------------------------ device exchange (xgmi) ---
void xs_set_timeout(gk_ctx *c, int ms) {
    c->xs_timeout_ms = ms;
    c->xs_timeout = (gk::u64)ms * (gk::u64)c->xs_tick_per_ms;
}

int xs_alloc(gk_ctx *c) {
    if (c->xs_buf != nullptr) return GK_OK;
    HIPCHK(hipSetDevice(c->dev));
    c->xs_words = gk::XS_RED_WORDS + 8LL * gk::XS_HALO_LINES * c->N;
    if (hipExtMallocWithFlags((void **)&c->xs_buf, sizeof(gk::u64) * c->xs_words, hipDeviceMallocUncached) !=
        hipSuccess)
        return set_err(GK_ERR_NOMEM, "cannot allocate the exchange region");
    HIPCHK(hipMemsetAsync(c->xs_buf, 0, sizeof(gk::u64) * c->xs_words, c->st));
    HIPCHK(hipMalloc((void **)&c->xs_seqdev, sizeof(unsigned)));
    HIPCHK(hipHostMalloc((void **)&c->xs_err, sizeof(int), hipHostMallocMapped));
    HIPCHK(hipHostGetDevicePointer((void **)&c->xs_err_dev, c->xs_err, 0));
    *c->xs_err = 0;
    int khz = 0;
    HIPCHK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, c->dev));
    if (khz > 0) c->xs_tick_per_ms = khz;
    xs_set_timeout(c, c->xs_timeout_ms);
    HIPCHK(hipStreamSynchronize(c->st));  // zeroed before any peer can see the region
    return GK_OK;
}

// The straggler named by a device-side failure code (gk::xs_fail).
std::string xs_culprit(int code) {
    const int op = code >> 16, src = (code & 0xFFFF) - 1;
    char buf[160];
    switch (op) {
        case gk::XSE_XCHG: std::snprintf(buf, sizeof buf, "rank %d's all-reduce granule", src); break;
        case gk::XSE_BCAST: std::snprintf(buf, sizeof buf, "rank %d's broadcast granule", src); break;
        case gk::XSE_HALO: std::snprintf(buf, sizeof buf, "the halo line of rank %d", src); break;
        case gk::XSE_RES_WG:
            std::snprintf(buf, sizeof buf, "workgroup %d of this rank inside a resident step (not co-resident?)", src);
            break;
        case gk::XSE_RES_RANK:
            std::snprintf(buf, sizeof buf, "rank %d's total inside a resident step (rank straggling)", src);
            break;
        default: std::snprintf(buf, sizeof buf, "an unknown peer (code %d)", code); break;
    }
    return buf;
}

// After a host wait: did a device exchange miss its deadline?  The exchange is
// then retired for the life of the context: sequence numbers may differ
// between ranks after a failed solve (a pipelined step was already queued), so
// its granules cannot be trusted again (gk_xchg_enable(1) refuses from now on)
// and resident steps go to the launch path.  The exchange is NOT switched off
// here: its error flag stays set, so every later exchange of this rank fails at
// once (NaN results, GK_ERR_COMM).  To continue, the CALLER switches every rank
// to RCCL / the local group with gk_xchg_enable(0) -- all ranks together, as
// bench.py's fallback does; flipping only the rank that saw the miss would
// desynchronise the ranks' collectives.
int xs_check(gk_ctx *c) {
    const int code = c->xs_err != nullptr ? __atomic_load_n(c->xs_err, __ATOMIC_ACQUIRE) : 0;
    if (code != 0) {
        c->xs_broken = true;
        c->res_broken = true;
        return set_err(GK_ERR_COMM, "device exchange: rank %d of %d missed the %d ms deadline waiting for %s",
                       c->rank, c->nranks, c->xs_timeout_ms, xs_culprit(code).c_str());
    }
    return GK_OK;
}

// After a host wait: did a resident step miss an in-launch deadline?  Then the
// context falls back to one launch per projection for the rest of its life.
int res_check(gk_ctx *c) {
    const int code = c->res_err != nullptr ? __atomic_load_n(c->res_err, __ATOMIC_ACQUIRE) : 0;
    if (code != 0) {
        *c->res_err = 0;
        c->res_broken = true;
        return set_err(GK_ERR_COMM,
                       "resident MGS-R step: an in-launch exchange missed its %d ms deadline waiting for %s; the "
                       "launch-per-projection path is used from now on",
                       c->res_timeout_ms, xs_culprit(code).c_str());
    }
    return GK_OK;
}

// Host-side watchdog of every wait on this context's stream: the device waits
// all carry deadlines, but a kernel that is never SCHEDULED (its queue not mapped:
// more processes / streams on a device than its hardware queues) would keep the
// host waiting forever.  Past twice the longest device deadline plus a minute,
// the wait fails with GK_ERR_COMM instead.
// GK_TUNE_WATCHDOG_MS overrides the limit (tests; a deployment that knows its queue drains).
long long watchdog_ms(const gk_ctx *c) {
    return c->watchdog_ms > 0 ? (long long)c->watchdog_ms : 2LL * std::max(c->res_timeout_ms, c->xs_timeout_ms) + 60000;
}

int spin_until(gk_ctx *c, hipError_t (*query)(void *), void *obj, const char *what) {
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned it = 1;; ++it) {
        const hipError_t r = query(obj);
        if (r == hipSuccess) return GK_OK;
        if (r != hipErrorNotReady) return set_err(GK_ERR_HIP, "%s: %s", what, hipGetErrorString(r));
        if ((it & 1023u) == 0) {
            const long long ms = std::chrono::duration_cast<std::chrono::milliseconds>(
                                     std::chrono::steady_clock::now() - t0).count();
            if (ms > watchdog_ms(c)) {
                // work is still queued on the stream: the context cannot be used (or its
                // buffers freed) safely any more -- every later call fails, gk_destroy
                // frees only once the stream has drained
                c->broken = true;
                return set_err(GK_ERR_COMM,
                               "%s: not complete after %lld ms (rank %d of %d): a kernel of this context was never "
                               "scheduled -- more streams on the device than hardware queues?  The context is broken.",
                               what, ms, c->rank, c->nranks);
            }
        }
    }
}

hipError_t query_stream(void *s) { return hipStreamQuery(static_cast<hipStream_t>(s)); }
hipError_t query_event(void *e) { return hipEventQuery(static_cast<hipEvent_t>(e)); }

int sync_st(gk_ctx *c) {
    CHK(spin_until(c, query_stream, c->st, "stream synchronize"));
    CHK(res_check(c));
    return xs_check(c);
}

int xs_exchange(gk_ctx *c, double *buf, int count, int mode, int root) {
    unsigned seq = ++c->xs_seq;
    const unsigned *base = nullptr;
    if (c->capturing) {  // a graph node: its number relative to the base set before each replay
        seq -= c->graph_seq0;
        base = c->xs_seqdev;
    }
    switch (mode) {
        case gk::XS_SLAB:
            gk::k_xchg<gk::XS_SLAB><<<1, gk::TPB, 0, c->st>>>(buf, count, c->xs_peers, c->nranks, c->rank, seq, base,
                                                            root, c->xs_err_dev, c->xs_timeout);
            break;
        case gk::XS_VEC:
            gk::k_xchg<gk::XS_VEC><<<1, gk::TPB, 0, c->st>>>(buf, count, c->xs_peers, c->nranks, c->rank, seq, base,
                                                           root, c->xs_err_dev, c->xs_timeout);
            break;
        default:
            gk::k_xchg<gk::XS_BCAST><<<1, gk::TPB, 0, c->st>>>(buf, count, c->xs_peers, c->nranks, c->rank, seq,
                                                             base, root, c->xs_err_dev, c->xs_timeout);
            break;
    }
    LAUNCHCHK();
    return GK_OK;
}

int lg_barrier(gk_ctx *c) {
    gk_group *g = c->lg;
    std::unique_lock<std::mutex> lk(g->mu);
    if (g->broken) return set_err(GK_ERR_STATE, "local group broken by an earlier timeout");
    const long my = g->gen;
    if (++g->arrived == g->n) {
        g->arrived = 0;
        ++g->gen;
        g->cv.notify_all();
        return GK_OK;
    }
    if (!g->cv.wait_for(lk, std::chrono::seconds(300), [&] { return g->gen != my || g->broken; }) || g->broken) {
        g->broken = true;
        g->cv.notify_all();
        return set_err(GK_ERR_STATE, "local group barrier timed out");
    }
    return GK_OK;
}

// Phase 1: publish `p` and an event after its producer; wait for everyone.
int lg_publish(gk_ctx *c, const double *p) {
    c->lg->ptrs[c->rank] = p;
    HIPCHK(hipEventRecord(c->lev_a, c->st));
    return lg_barrier(c);
}

int lg_wait(gk_ctx *c, int q, bool second) {
    gk_ctx *o = c->lg->members[q];
    HIPCHK(hipStreamWaitEvent(c->st, second ? o->lev_b : o->lev_a, 0));
    return GK_OK;
}

// `vec`: element-wise sum of a short vector; otherwise `buf` is a partial slab
// whose consumer re-reduces it (any split of the same total is equivalent).
int allreduce(gk_ctx *c, double *buf, int count, bool vec = false) {
    if (!collective(c)) return GK_OK;
    ProfScope ps(c, GK_KID_COMM);
    if (c->xs_on) {
        if (!vec) return xs_exchange(c, buf, count, gk::XS_SLAB, 0);
        for (int k0 = 0; k0 < count; k0 += gk::XS_MAXV)
            CHK(xs_exchange(c, buf + k0, std::min(gk::XS_MAXV, count - k0), gk::XS_VEC, 0));
        return GK_OK;
    }
    if (c->lg == nullptr) {
        NCCLCHK(ncclAllReduce(buf, buf, count, ncclDouble, ncclSum, c->comm, c->st));
        return GK_OK;
    }
    if (count > gk::NPMAX * 4) return set_err(GK_ERR_ARG, "local allreduce too large");
    CHK(lg_publish(c, buf));
    RankPtrs rp{};
    for (int q = 0; q < c->nranks; ++q) {
        CHK(lg_wait(c, q, false));
        rp.p[q] = c->lg->ptrs[q];
    }
    k_sum_ranks<<<(count + 255) / 256, 256, 0, c->st>>>(rp, c->nranks, c->lscratch, count);
    LAUNCHCHK();
    HIPCHK(hipEventRecord(c->lev_b, c->st));
    CHK(lg_barrier(c));
    for (int q = 0; q < c->nranks; ++q) CHK(lg_wait(c, q, true));  // nobody reads buf any more
    HIPCHK(hipMemcpyAsync(buf, c->lscratch, sizeof(double) * count, hipMemcpyDeviceToDevice, c->st));
    return GK_OK;
}

int bcast(gk_ctx *c, double *buf, int count, int root) {
    if (!collective(c)) return GK_OK;
    ProfScope ps(c, GK_KID_COMM);
    if (c->xs_on) {
        for (int k0 = 0; k0 < count; k0 += gk::XS_MAXV)
            CHK(xs_exchange(c, buf + k0, std::min(gk::XS_MAXV, count - k0), gk::XS_BCAST, root));
        return GK_OK;
    }
    if (c->lg == nullptr) {
        NCCLCHK(ncclBroadcast(buf, buf, count, ncclDouble, root, c->comm, c->st));
        return GK_OK;
    }
    CHK(lg_publish(c, buf));
    if (c->rank != root) {
        CHK(lg_wait(c, root, false));
        HIPCHK(hipMemcpyAsync(buf, c->lg->ptrs[root], sizeof(double) * count, hipMemcpyDeviceToDevice, c->st));
    }
    HIPCHK(hipEventRecord(c->lev_b, c->st));
    CHK(lg_barrier(c));
    if (c->rank == root)
        for (int q = 0; q < c->nranks; ++q) CHK(lg_wait(c, q, true));
    return GK_OK;
}

// Exchange nl grid lines of vec with the slab neighbours: lo <- the last nl
// lines of rank-1 (our rows -nl..-1), hi <- the first nl lines of rank+1 (our
// rows nlines..nlines+nl-1).  nl = 1 for a stencil sweep; the temporal-blocked
// Chebyshev passes need nl = L (their recompute cone).
int halo_lines(gk_ctx *c, const double *vec, int nl, double *lo, double *hi) {
    if (!collective(c)) return GK_OK;
    // a slab thinner than the halo would send lines it does not own (and its
    // neighbours would need lines from two ranks away)
    if (c->nranks > 1 && (nl < 1 || nl > c->nlines))
        return set_err(GK_ERR_ARG, "halo of %d lines from a slab of %d lines (rank %d)", nl, c->nlines, c->rank);
    ProfScope ps(c, GK_KID_HALO);
    const int N = c->N;
    const i64 cnt = (i64)nl * N;
    if (c->xs_on) {
        if (c->nranks == 1) return GK_OK;
        const unsigned seq = ++c->xs_hseq;
        gk::k_xhalo<<<(unsigned)((cnt + gk::TPB - 1) / gk::TPB), gk::TPB, 0, c->st>>>(
            vec, N, c->nlines, nl, c->xs_peers, c->nranks, c->rank, seq, lo, hi, c->xs_err_dev, c->xs_timeout);
        LAUNCHCHK();
        return GK_OK;
    }
    if (c->lg == nullptr) {
        NCCLCHK(ncclGroupStart());
        if (c->rank > 0) {
            NCCLCHK(ncclSend(vec, cnt, ncclDouble, c->rank - 1, c->comm, c->st));
            NCCLCHK(ncclRecv(lo, cnt, ncclDouble, c->rank - 1, c->comm, c->st));
        }
        if (c->rank < c->nranks - 1) {
            NCCLCHK(ncclSend(vec + (i64)(c->nlines - nl) * N, cnt, ncclDouble, c->rank + 1, c->comm, c->st));
            NCCLCHK(ncclRecv(hi, cnt, ncclDouble, c->rank + 1, c->comm, c->st));
        }
        NCCLCHK(ncclGroupEnd());
        return GK_OK;
    }
    CHK(lg_publish(c, vec));
    if (c->rank > 0) {
        gk_ctx *o = c->lg->members[c->rank - 1];
        CHK(lg_wait(c, c->rank - 1, false));
        HIPCHK(hipMemcpyAsync(lo, c->lg->ptrs[c->rank - 1] + (i64)(o->nlines - nl) * N, sizeof(double) * cnt,
                              hipMemcpyDeviceToDevice, c->st));
    }
    if (c->rank < c->nranks - 1) {
        CHK(lg_wait(c, c->rank + 1, false));
        HIPCHK(hipMemcpyAsync(hi, c->lg->ptrs[c->rank + 1], sizeof(double) * cnt, hipMemcpyDeviceToDevice, c->st));
    }
    HIPCHK(hipEventRecord(c->lev_b, c->st));
    CHK(lg_barrier(c));
    if (c->rank > 0) CHK(lg_wait(c, c->rank - 1, true));
    if (c->rank < c->nranks - 1) CHK(lg_wait(c, c->rank + 1, true));
    return GK_OK;
}

int halo(gk_ctx *c, const double *vec) { return halo_lines(c, vec, 1, c->hlo, c->hhi); }

const double *halo_lo(gk_ctx *c) { return (c->nranks > 1 && c->rank > 0) ? c->hlo : nullptr; }
const double *halo_hi(gk_ctx *c) { return (c->nranks > 1 && c->rank < c->nranks - 1) ? c->hhi : nullptr; }

// -------------------------------------------------------------- geometry ---
bool nt_auto_for(i64 max_nloc);

void set_geometry(gk_ctx *c) {
    const int N = c->N;
    c->vec = (N % 2 == 0) ? 2 : 1;
    const int gx = (N + gk::TPB * c->vec - 1) / (gk::TPB * c->vec);
    const int ml = c->max_lines > 0 ? c->max_lines : c->nlines;
    // ~2048 workgroups for the stencil sweeps, marching JT lines each
    const int target = c->tune_st_blocks > 0 ? c->tune_st_blocks : 2048;
    int JT = (int)std::max<i64>(1, ((i64)ml * gx + target - 1) / target);
    if (JT > 64) JT = 64;
    int gy = (ml + JT - 1) / JT;
    while ((i64)gx * gy > gk::NPMAX) {
        ++JT;
        gy = (ml + JT - 1) / JT;
    }
    c->JT = JT;
    c->sgrid = dim3(gx, gy, 1);
    c->np_st = gx * gy;
    {  // the short-recurrence marches: fewer, longer marches (each re-reads 2 neighbour lines per march)
        const int srt = c->tune_sr_blocks > 0 ? c->tune_sr_blocks : 512;
        int sjt = (int)std::max<i64>(1, ((i64)ml * gx + srt - 1) / srt);
        if (sjt > 256) sjt = 256;
        int sgy = (ml + sjt - 1) / sjt;
        while ((i64)gx * sgy > gk::NPMAX) {
            ++sjt;
            sgy = (ml + sjt - 1) / sjt;
        }
        c->sr_JT = sjt;
        c->sr_sgrid = dim3(gx, sgy, 1);
        c->np_sr = gx * sgy;
    }
    // projection kernels: fixed workgroup count derived from the largest slab
    const i64 nmax2 = ((i64)ml * N + 1) / 2;
    i64 npj = (nmax2 + (i64)gk::TPB * gk::UNR - 1) / ((i64)gk::TPB * gk::UNR);
    if (npj > 1024) npj = 1024;
    if (c->tune_pj_blocks > 0) npj = std::min<i64>(c->tune_pj_blocks, gk::NPMAX);
    // Krylov columns by non-temporal loads once a vector no longer fits
    // comfortably beside them in the 256 MiB Infinity Cache (measured: -20 %
    // projection time at 4096^2, +6 % at 1024^2 where everything is resident).
    c->nt_auto = nt_auto_for((i64)ml * N);
    if (npj < 1) npj = 1;
    c->np_pj = (int)npj;
    // elementwise kernels: also from the largest slab (their partial slabs are all-reduced)
    i64 nb = (nmax2 + gk::TPB - 1) / gk::TPB;
    c->nblk_stream = (int)std::min<i64>(std::max<i64>(nb, 1), 2048);
}

// -------------------------------------------------------------- launches ---
template <int VEC, int OP, int ACC>
int launch_stencil_v(gk_ctx *c, const gk::StArgs &a) {
    gk::k_stencil<VEC, OP, ACC><<<c->sgrid, gk::TPB, 0, c->st>>>(a);
    LAUNCHCHK();
    return GK_OK;
}

template <int OP, int ACC>
int launch_stencil_o(gk_ctx *c, const gk::StArgs &a) {
    return c->vec == 2 ? launch_stencil_v<2, OP, ACC>(c, a) : launch_stencil_v<1, OP, ACC>(c, a);
}

template <int OP>
int launch_stencil_a(gk_ctx *c, int acc, const gk::StArgs &a) {
    if (acc == gk::ACC_NONE) return launch_stencil_o<OP, gk::ACC_NONE>(c, a);
    if (acc == gk::ACC_DOT) return launch_stencil_o<OP, gk::ACC_DOT>(c, a);
    return launch_stencil_o<OP, gk::ACC_NORM>(c, a);
}

int stencil(gk_ctx *c, int op, int acc, gk::StArgs a) {
    ProfScope ps(c, GK_KID_STENCIL);
    if (acc != gk::ACC_NONE) c->last_np = c->np_st;
    a.hlo = halo_lo(c);
    a.hhi = halo_hi(c);
    a.N = c->N;
    a.nlines = c->nlines;
    a.JT = c->JT;
    switch (op) {
        case gk::OP_PLAIN: return launch_stencil_a<gk::OP_PLAIN>(c, acc, a);
        case gk::OP_RESID: return launch_stencil_a<gk::OP_RESID>(c, acc, a);
        case gk::OP_CBPR2: return launch_stencil_a<gk::OP_CBPR2>(c, acc, a);
        case gk::OP_CHEB_FIRST: return launch_stencil_a<gk::OP_CHEB_FIRST>(c, acc, a);
        default: return launch_stencil_a<gk::OP_CHEB_ITER>(c, acc, a);
    }
}

template <bool NT, int U>
void launch_proj_u(gk_ctx *c, int mode, double *w, const double *va, const double *vb, const double *pin,
                   int npin, double *pout, double *hslot, double coef, i64 tail0, int hstore) {
    const dim3 g(c->np_pj);
    const i64 n = c->nloc;
    const int bl = c->tune_blocked;
    switch (mode) {
        case gk::PJ_DOT:
            gk::k_proj<gk::PJ_DOT, NT, U><<<g, gk::TPB, 0, c->st>>>(w, va, vb, pin, npin, pout, hslot, coef, n,
                                                                    tail0, bl, hstore);
            break;
        case gk::PJ_AXPY:
            gk::k_proj<gk::PJ_AXPY, NT, U><<<g, gk::TPB, 0, c->st>>>(w, va, vb, pin, npin, pout, hslot, coef, n,
                                                                     tail0, bl, hstore);
            break;
        case gk::PJ_AXPY_DOT:
            gk::k_proj<gk::PJ_AXPY_DOT, NT, U><<<g, gk::TPB, 0, c->st>>>(w, va, vb, pin, npin, pout, hslot, coef,
                                                                         n, tail0, bl, hstore);
            break;
        default:
            gk::k_proj<gk::PJ_AXPY_NORM, NT, U><<<g, gk::TPB, 0, c->st>>>(w, va, vb, pin, npin, pout, hslot, coef,
                                                                          n, tail0, bl, hstore);
            break;
    }
}

template <bool NT>
void launch_proj(gk_ctx *c, int mode, double *w, const double *va, const double *vb, const double *pin,
                 int npin, double *pout, double *hslot, double coef, i64 tail0, int hstore) {
    int u = c->tune_unr;
    if (u == 0) {  // auto: one trip per thread when the vector is small, else 2 in flight
        const i64 per_thread = (c->nloc / 2 + (i64)c->np_pj * gk::TPB - 1) / ((i64)c->np_pj * gk::TPB);
        u = per_thread <= 4 ? 4 : 2;
    }
    if (u == 2)
        launch_proj_u<NT, 2>(c, mode, w, va, vb, pin, npin, pout, hslot, coef, tail0, hstore);
    else if (u == 8)
        launch_proj_u<NT, 8>(c, mode, w, va, vb, pin, npin, pout, hslot, coef, tail0, hstore);
    else
        launch_proj_u<NT, 4>(c, mode, w, va, vb, pin, npin, pout, hslot, coef, tail0, hstore);
}

int proj(gk_ctx *c, int mode, double *w, const double *va, const double *vb, const double *pin,
         int npin, double *pout, double *hslot, double coef, i64 tail0 = 0, int hstore = 0) {
    ProfScope ps(c, GK_KID_PROJ);
    if (c->tune_nt > 0 || (c->tune_nt < 0 && c->nt_auto))
        launch_proj<true>(c, mode, w, va, vb, pin, npin, pout, hslot, coef, tail0, hstore);
    else
        launch_proj<false>(c, mode, w, va, vb, pin, npin, pout, hslot, coef, tail0, hstore);
    LAUNCHCHK();
    return GK_OK;
}

int scale(gk_ctx *c, double *out, const double *w, const double *pin, int npin, double *hslot,
          double *hcopy = nullptr, const double *hsrc = nullptr, int ncopy = 0, bool pin_norm = false) {
    ProfScope ps(c, GK_KID_SCALE);
    gk::k_scale<<<c->nblk_stream, gk::TPB, 0, c->st>>>(out, w, pin, npin, hslot, c->nloc, hcopy, hsrc, ncopy,
                                                       pin_norm ? 1 : 0);
    LAUNCHCHK();
    return GK_OK;
}

// NORM2 of x(0:n) in flang-rt's order into out[0] (GK_TUNE_HH_NORM_ORDER)
int norm2_seq(gk_ctx *c, const double *x, i64 n, double *out) {
    ProfScope ps(c, GK_KID_OTHER);
    gk::k_norm2_seq<<<1, gk::TPB, 0, c->st>>>(x, n, out);
    LAUNCHCHK();
    return GK_OK;
}

int finalize(gk_ctx *c, const double *pin, int npin, double *out, int take_sqrt) {
    ProfScope ps(c, GK_KID_OTHER);
    gk::k_finalize<<<1, gk::TPB, 0, c->st>>>(pin, npin, out, take_sqrt);
    LAUNCHCHK();
    return GK_OK;
}

// ------------------------------------------------ resident MGS-R step ----
constexpr int RES_LDS_MIN = 96 * 1024;  // dynamic LDS: > half a CU's 160 KiB, so one workgroup per CU
constexpr int RES_L2 = 18;              // LDS-resident double2 of w per data thread (18 x 512 x 16 B = 144 KiB)
constexpr int RES_R2_BIG = 12;          // two register arrays of 12 double2 fit 256 VGPRs without spills

#ifndef GK_RES_RW
#define GK_RES_RW 89
#endif
#ifndef GK_RES_LW
#define GK_RES_LW 39
#endif
// w-only variant: double2 of w per thread in registers / LDS.  The MGS step holds 89 + 39
// chunks -- the whole 4096^2 slab on chip, nothing streamed -- since round 5 sized its H
// column in LDS by m (gk::WO_HMAX) instead of RHMAX; rounds 1-4 held 88 + 38 and streamed
// 1.5 % of w at 32 B per unknown.  The reflection chains keep 90 + 38 (RES_RW_HH, RES_LW_HH).
constexpr int RES_RW = GK_RES_RW, RES_LW = GK_RES_LW, RES_LW_HH = 38;
#ifndef GK_RES_RW_HH
#define GK_RES_RW_HH 90
#endif
// The reflection chains hold two chunks more (RW 90 with a 6-deep batch: 90 + 38 chunks =
// the whole 4096^2 slab on chip, nothing streamed): A/B at 4096^2 (profiles/r02/ab_rw_hh.jsonl)
// Householder 41.05 -> 40.57 us per reflection, while the MGS-R step keeps 88 / 8 (41.2 vs
// 41.67 us with 90 / 6).
constexpr int RES_RW_HH = GK_RES_RW_HH;

struct ResPlan {
    int G = 0, r2 = 0, l2 = 0;
    int r2e = 0, l2e = 0;  // chunks per workgroup used: the resident prefix spread evenly over G
    bool pf = false, nt = false, cw = false, wo = false;
    bool pc = false;       // column-cache variant (k_mgs_wpc): w in registers, running column cached
    bool pcs = false;      // ... its 16-chunk instantiation (whole column in registers)
    int blk = 0;           // > 1: the blocked-projection MGS step k_mgs_blk with blocks of `blk` (gk_blk.hpp);
                           // 1 with bvar >= 0: the strict step on k_mgs_blk<S = 1> (GK_TUNE_RES_PF)
    int bvar = -1;         // ... its instantiation (gk::BLK_*)
    int wt = 0;            // threads per workgroup = double2 per chunk (set by plan_resident)
    i64 nres2 = 0;
    int lds = 0;
};

// Column-cache variant (k_mgs_wpc): w of up to RES_PC_RW chunks per thread in
// registers, the running column of RES_PC_RX of them in registers and of
// RES_PC_LX in LDS; a pass streams its dot column in batches of WB chunks.
// PC_NT = threads per workgroup.  512 (default, two waves per SIMD: one wave's
// batch is in flight while the other consumes its own): 32 chunks of w per
// thread, 4 + 19 of the column cached (the 9 others read V_i too: 10.25 B per
// unknown at 2896^2), batches of 4; at 2896^2 15.5 us per projection against 17.6
// for the one-wave build (profiles/r04/ab_pc512_r04j.jsonl) -- 13 + 19 cached spill
// at 256 VGPRs per wave (the two-wave budget).  256 (one wave per SIMD, the first
// build): 64 chunks per thread, 26 + 38 cached (8 B per unknown), batches of 8
// (4, 16 and a software-pipelined 8 were slower, ab_wpc_r04c/d), 6 for the
// reflection chains.  PC_TOUCH > 0 touches the first chunks of the next pass's dot
// column into L2 during each all-gather: on the one-wave build it shortened the
// pass and lengthened the wait by as much (2896^2: touch 28 / 16 / 0 -> 18.2 /
// 17.8 / 17.6 us per projection, ab_wpc_touch_r04e), so it is off.
#ifndef GK_RES_PC_NT
#define GK_RES_PC_NT 512
#endif
#ifndef GK_RES_PC_WB
#define GK_RES_PC_WB (GK_RES_PC_NT == 512 ? 4 : 8)
#endif
#ifndef GK_RES_PC_WB_HH
#define GK_RES_PC_WB_HH (GK_RES_PC_NT == 512 ? 4 : 6)
#endif
#ifndef GK_RES_PC_TOUCH
#define GK_RES_PC_TOUCH 0
#endif
#ifndef GK_RES_PC_RX
#define GK_RES_PC_RX (GK_RES_PC_NT == 512 ? 4 : 26)
#endif
constexpr int RES_PC_NT = GK_RES_PC_NT;
static_assert(RES_PC_NT == 256 || RES_PC_NT == 512, "column-cache workgroups of one or two waves per SIMD");
#ifndef GK_RES_PC_RX_MGS
#define GK_RES_PC_RX_MGS (GK_RES_PC_NT == 512 ? 6 : GK_RES_PC_RX)
#endif
// RX_MGS: the MGS step's register-cached chunks (6 fit its register budget; the
// reflection chains spill 20 B per lane at 6 and keep RX = 4)
constexpr int RES_PC_RW = RES_PC_NT == 512 ? 32 : 64, RES_PC_RX = GK_RES_PC_RX, RES_PC_LX = RES_PC_NT == 512 ? 19 : 38;
constexpr int RES_PC_RX_MGS = GK_RES_PC_RX_MGS;
constexpr int RES_PC_WB = GK_RES_PC_WB, RES_PC_WB_HH = GK_RES_PC_WB_HH, RES_PC_TOUCH = GK_RES_PC_TOUCH;
// Slabs of at most 16 chunks per thread (two-wave build): k_mgs_wpc<16, 16, 0> -- w and
// its whole column in registers, no LDS, half the unrolled pass of the 32-chunk kernel.
#ifndef GK_RES_PC_SMALL
#define GK_RES_PC_SMALL 1
#endif
constexpr bool RES_PCS = GK_RES_PC_SMALL != 0 && RES_PC_NT == 512;
constexpr int RES_PCS_RW = 16, RES_PCS_RX = 16, RES_PCS_LX = 0;

// Modelled bytes per projection of a slab of n2 double2 on G workgroups (the
// unit of pairs_bytes / wonly_bytes: 8 per double2 whose w and running column are
// on chip, 16 per double2 of w alone, 32 per streamed double2) under the
// column-cache variant: the cached pairs, the rest of the register-held w, the
// streamed rest.
i64 pc_bytes(i64 n2, int G, bool hh) {
    if (RES_PCS && n2 <= (i64)G * RES_PCS_RW * RES_PC_NT) return 8 * n2;  // the 16-chunk kernel: all cached
    const int rx = hh ? RES_PC_RX : RES_PC_RX_MGS;
    const i64 cap = (i64)G * RES_PC_RW * RES_PC_NT, cached = (i64)G * (rx + RES_PC_LX) * RES_PC_NT;
    const i64 r = std::min(n2, cap), c = std::min(r, cached);
    return 8 * c + 16 * (r - c) + 32 * (n2 - r);
}

// Modelled fabric bytes per projection (per double2) of the two large-slab
// variants: pairs (w + running column, 8 B/unknown) in 2 x 12 registers + w in
// LDS (16 B) vs w only in registers + LDS (16 B); the rest streams (32 B).
i64 pairs_bytes(i64 n2, int G) {  // k_mgs_res<12, 18>: 2 x 12 registers + 18 LDS chunks of w
    const i64 rp = (i64)G * RES_R2_BIG * gk::RT, lp = (i64)G * RES_L2 * gk::RT;
    auto clamp = [](i64 v) { return v < 0 ? (i64)0 : v; };
    const i64 pr = std::min(n2, rp), pl = std::min(clamp(n2 - rp), lp), ps = clamp(n2 - rp - lp);
    return 8 * pr + 16 * pl + 32 * ps;
}

i64 wonly_bytes(i64 n2, int G) {
    const i64 rw = (i64)G * (RES_RW + RES_LW) * gk::WT;  // (the MGS step's; the reflection chains' is the same 128)
    const i64 wr = std::min(n2, rw), ws = n2 > rw ? n2 - rw : 0;
    return 16 * wr + 32 * ws;
}

bool wonly_pays(i64 n2, int G) { return wonly_bytes(n2, G) < pairs_bytes(n2, G); }

// The variant a slab of nloc local unknowns runs on (pure: no context, no
// device; gk_res_plan_query exposes it so the CPU tests pin what every
// production split selects).
//   fits in 3 x R2 <= 8 registers (w, running column, prefetched column) with
//   wave 0 kept for the exchange: R2 in {2,4,8}, PF + CW;
//   else w only in registers + LDS when the byte model says so (GK_TUNE_RES_WONLY);
//   else w and the running column in 2 x 12 registers, plus (GK_TUNE_RES_LDS)
//   w of 18 more chunks per workgroup in LDS, the rest streamed.
void plan_resident(i64 nloc, int gmax, int cap, int tune_lds, int tune_wonly, bool hh, bool nt, ResPlan &p,
                   int tune_pc = -1, int tune_blk = 1, int tune_pf = 0) {
    const i64 n2 = nloc / 2;
    const i64 dcw = gk::RT - 64;
    // small vectors: no more workgroups than two chunks each (a cheaper all-gather)
    const int gcw = (int)std::max<i64>(1, std::min<i64>(gmax, (n2 + 2 * dcw - 1) / (2 * dcw)));
    const i64 need = (n2 + (i64)gcw * dcw - 1) / ((i64)gcw * dcw);
    p = ResPlan{};
    static const int pfs[] = {2, 4, 8};
    for (int s : pfs)
        if (s <= cap && (p.r2 == 0 || p.r2 < need)) p.r2 = s;
    // Spread the resident chunks evenly: every workgroup holds ceil(chunks / G)
    // register chunks (at most the variant's R), then the same for LDS -- a
    // contiguous fill would leave the last workgroups idle and make the first
    // ones set the pace of every all-gather (2048^2: slowest pass 10.2 us vs
    // 4.3 us median).
    auto spread = [&](i64 dt, int rmax, int lmax) {
        const i64 nchf = n2 / dt, G = p.G;
        p.r2e = (int)std::min<i64>(rmax, (nchf + G - 1) / G);
        const i64 rest = std::max<i64>(0, nchf - G * p.r2e);
        p.l2e = (int)std::min<i64>(lmax, (rest + G - 1) / G);
        p.nres2 = std::min<i64>(nchf, G * (p.r2e + p.l2e)) * dt;
    };
    // The column-cache variant where it moves fewer bytes than both large-slab
    // variants.  The two-wave build streams as fast as k_mgs_res (2896^2: 10.25 vs
    // 14 B/unknown -> 15.5 vs 18.8 us per projection; 2048^2: 8 vs 10 -> 8.8 vs 9.6,
    // profiles/r04/ab_pc512_r04j.jsonl).  The one-wave build streamed at ~4.7 TB/s
    // to k_mgs_res's ~6.8, so there it had to save a third of the bytes (2048^2 was
    // slower on it: 11.3-11.5 vs 9.6 us, ab_wpc_touch_r04e).
    const int var = gk::blk_variant((n2 + (i64)gmax * 512 - 1) / ((i64)gmax * 512));
    // The strict step on k_mgs_blk<S = 1> (the next dot column prefetched into LDS during each
    // all-gather), opt-in (GK_TUNE_RES_PF 1) for slabs up to 32 chunks of 512.  Faster than the
    // strict kernels only at 16 chunks on one GPU (2048^2 8.04 -> 7.64 us per projection;
    // 1024^2 3.78 -> 4.33, 1448^2 5.67 -> 5.77, 2896^2 15.0 -> 20.5: profiles/r05/
    // ab_strict_pf_r05w.txt), and at the load it helps -- the 4096^2 / 4 split -- the 4-rank
    // same-device rehearsal ran slower on it (1,061 vs 1,110 it/s, its all-gather wait 3.9 ->
    // 7.6 us: reh4_2048_pf_r05x.json vs reh4_2048_r05z.json), so it is not the default.
    const bool pf = !hh && tune_blk == 1 && var != gk::BLK_WONLY && tune_pf > 0;
    if (!hh && (tune_blk > 1 || pf)) {
        // the blocked-projection MGS step (opt-in): the instantiation by the chunks of
        // 512 double2 a workgroup holds -- w in registers (+ LDS for the w-only build)
        // and blocks of S columns cached where they fit (gk_blk.hpp); S = 1
        // (GK_TUNE_RES_PF): the strict step on the same kernel and its LDS prefetch
        p.G = gmax;
        const gk::BlkGeom g = gk::blk_geom(var, tune_blk);
        p.blk = tune_blk;
        p.bvar = var;
        p.wt = g.nt;
        spread(g.nt, g.rw, g.lw);
        p.r2 = g.rx;
        p.l2 = g.lx;
        p.lds = (g.lw + tune_blk * (g.lx + g.pfx)) * g.nt * (int)sizeof(double2);
        p.nt = true;
        return;
    }
    const bool pc_fits = n2 <= (i64)gmax * RES_PC_RW * RES_PC_NT;
    const i64 other_bytes = std::min(pairs_bytes(n2, gmax), wonly_bytes(n2, gmax));
    const bool pc_pays = pc_fits && (RES_PC_NT == 512 ? pc_bytes(n2, gmax, hh) < other_bytes
                                                      : 3 * pc_bytes(n2, gmax, hh) <= 2 * other_bytes);
    if (p.r2 >= need || cap < RES_R2_BIG) {
        p.G = gcw;
        p.pf = p.cw = true;
        spread(dcw, p.r2, 0);
    } else if (tune_wonly <= 0 && (tune_pc > 0 ? pc_fits : (tune_pc < 0 && pc_pays))) {
        // w wholly in registers, the running column cached (k_mgs_wpc): 8 B/unknown
        p.G = gmax;
        p.pc = true;
        p.wt = RES_PC_NT;
        spread(RES_PC_NT, RES_PC_RW, 0);
        p.pcs = RES_PCS && p.r2e <= RES_PCS_RW;
        p.r2 = p.pcs ? RES_PCS_RX : (hh ? RES_PC_RX : RES_PC_RX_MGS);
        p.l2 = p.pcs ? RES_PCS_LX : RES_PC_LX;
        p.lds = p.l2 * RES_PC_NT * (int)sizeof(double2);
        p.nt = true;
        return;
    } else if (tune_wonly > 0 || (tune_wonly < 0 && wonly_pays(n2, gmax))) {
        // w only, one wave per SIMD: 16 B/unknown per projection for ~100 chunks per workgroup
        p.G = gmax;
        p.wo = true;
        p.wt = gk::WT;
        p.r2 = 0;  // (the kernel's register part is RES_RW / RES_RW_HH chunks: r2e)
        spread(gk::WT, hh ? RES_RW_HH : RES_RW, hh ? RES_LW_HH : RES_LW);
        p.lds = (hh ? RES_LW_HH : RES_LW) * gk::WT * (int)sizeof(double2);
        p.nt = true;  // V_i non-temporal, V_q default policy (fixed in the kernel)
        return;
    } else {
        p.G = gmax;
        p.r2 = RES_R2_BIG;
        const i64 dt = gk::RT, regs = (i64)p.G * RES_R2_BIG * dt;
        p.l2 = (tune_lds && n2 / dt * dt > regs) ? RES_L2 : 0;
        spread(dt, RES_R2_BIG, p.l2);
    }
    p.lds = std::max<int>(RES_LDS_MIN, p.l2 * (p.cw ? gk::RT - 64 : gk::RT) * (int)sizeof(double2));
    p.wt = gk::RT;
    p.nt = nt;
}

// Non-temporal Krylov-column loads once a vector of the largest slab no longer
// fits comfortably beside them in the 256 MiB Infinity Cache (set_geometry).
bool nt_auto_for(i64 max_nloc) { return max_nloc * 8 > (i64)48 * 1024 * 1024; }

// Can step j run as one resident launch, and with which variant?  Needs an
// in-launch reduction path: single rank, or the device exchange (RCCL and the
// host-side local group cannot be driven from inside a kernel).
bool res_plan(gk_ctx *c, ResPlan &p, bool hh = false) {
    if (c->tune_res == 0 || c->res_broken || c->m > gk::RHMAX || c->res_cus <= 0 || c->res_gath == nullptr)
        return false;
    if (collective(c) && !(c->xs_on && c->nranks > 1)) return false;
    // Several resident launches on one device spin on each other's partials, so
    // their streams must run concurrently -- HIP promises nothing about how
    // streams map to hardware queues.  Auto mode assumes one context per device.
    if (c->tune_res < 0 && c->res_share > 1) return false;
    const int gmax = std::max(1, std::min(gk::RGMAX, c->res_cus / std::max(1, c->res_share)));
    const int cap = c->tune_res_r2 > 0 ? c->tune_res_r2 : RES_R2_BIG;
    plan_resident(c->nloc, gmax, cap, c->tune_res_lds, c->tune_res_wonly, hh,
                  c->tune_nt > 0 || (c->tune_nt < 0 && c->nt_auto), p, c->tune_res_pc, c->tune_res_blk, c->tune_res_pf);
    if (p.wo && !hh && c->m + 1 > gk::WO_HMAX) return false;  // its H column: WO_HMAX entries of LDS
    return true;
}

// gk_res_plan_query / gk_res_info layout
enum { RPI_VARIANT = 0, RPI_G, RPI_R2, RPI_L2, RPI_PF, RPI_CW, RPI_WO, RPI_NT, RPI_R2E, RPI_L2E, RPI_LDS, RPI_NRES2, RPI_UNUSED12,
       RPI_CHEB_STEN, RPI_WT, RPI_BLK };
void plan_info(const ResPlan &p, bool on, long long *info) {
    for (int k = 0; k < GK_RES_INFO_LEN; ++k) info[k] = 0;
    if (!on) return;
    info[RPI_VARIANT] = p.bvar >= 0 ? GK_RES_BLOCKED
                        : p.pc    ? GK_RES_WCOL
                                  : (p.wo ? GK_RES_WONLY
                                          : (p.pf ? GK_RES_PREFETCH : (p.l2 > 0 ? GK_RES_PAIRS_LDS : GK_RES_PAIRS)));
    info[RPI_BLK] = p.bvar >= 0 ? p.blk : 1;
    info[RPI_G] = p.G;
    info[RPI_R2] = p.r2;
    info[RPI_L2] = p.l2;
    info[RPI_PF] = p.pf;
    info[RPI_CW] = p.cw;
    info[RPI_WO] = p.wo;
    info[RPI_NT] = p.nt;
    info[RPI_R2E] = p.r2e;
    info[RPI_L2E] = p.l2e;
    info[RPI_LDS] = p.lds;
    info[RPI_NRES2] = p.nres2;
    info[RPI_WT] = p.wt;
}

// hipFuncSetAttribute is per device: remember the dynamic-LDS size set on each.
constexpr int ATTR_DEVS = 64;

template <int R2, int L2, bool PF, bool NT, bool CW, int MODE>
int launch_res_m(gk_ctx *c, const ResPlan &p, const gk::ResArgs &a) {
    static std::atomic<int> attr[ATTR_DEVS];
    if (c->dev < 0 || c->dev >= ATTR_DEVS) return set_err(GK_ERR_ARG, "device id %d out of range", c->dev);
    if (attr[c->dev].load() < p.lds) {
        HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void *>(&gk::k_mgs_res<R2, L2, PF, NT, CW, MODE>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, p.lds));
        attr[c->dev] = p.lds;
    }
    gk::k_mgs_res<R2, L2, PF, NT, CW, MODE><<<p.G, gk::RT, p.lds, c->st>>>(a);
    LAUNCHCHK();
    return GK_OK;
}

template <int R2, int L2, bool PF, bool NT, bool CW>
int launch_res_t(gk_ctx *c, const ResPlan &p, const gk::ResArgs &a) {
    switch (a.mode) {
        case gk::RES_HH_UP: return launch_res_m<R2, L2, PF, NT, CW, gk::RES_HH_UP>(c, p, a);
        case gk::RES_HH_DOWN: return launch_res_m<R2, L2, PF, NT, CW, gk::RES_HH_DOWN>(c, p, a);
        default: return launch_res_m<R2, L2, PF, NT, CW, gk::RES_MGS>(c, p, a);
    }
}

template <int MODE>
int launch_wres_m(gk_ctx *c, const ResPlan &p, const gk::ResArgs &a) {
    constexpr int RW = MODE == gk::RES_MGS ? RES_RW : RES_RW_HH;
    constexpr int LW = MODE == gk::RES_MGS ? RES_LW : RES_LW_HH;
    constexpr int WBT = MODE == gk::RES_MGS ? gk::WB : gk::WB_HH;
    static std::atomic<int> attr[ATTR_DEVS];
    if (c->dev < 0 || c->dev >= ATTR_DEVS) return set_err(GK_ERR_ARG, "device id %d out of range", c->dev);
    if (attr[c->dev].load() < p.lds) {
        HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void *>(&gk::k_mgs_wres<RW, LW, MODE, WBT>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, p.lds));
        attr[c->dev] = p.lds;
    }
    gk::k_mgs_wres<RW, LW, MODE, WBT><<<p.G, gk::WT, p.lds, c->st>>>(a);
    LAUNCHCHK();
    return GK_OK;
}

int launch_wres(gk_ctx *c, const ResPlan &p, const gk::ResArgs &a) {
    switch (a.mode) {
        case gk::RES_HH_UP: return launch_wres_m<gk::RES_HH_UP>(c, p, a);
        case gk::RES_HH_DOWN: return launch_wres_m<gk::RES_HH_DOWN>(c, p, a);
        default: return launch_wres_m<gk::RES_MGS>(c, p, a);
    }
}

template <int RW, int RX, int LX, int MODE>
int launch_wpc_k(gk_ctx *c, const ResPlan &p, const gk::ResArgs &a) {
    constexpr int WBT = MODE == gk::RES_MGS ? RES_PC_WB : RES_PC_WB_HH;
    static std::atomic<int> attr[ATTR_DEVS];
    if (c->dev < 0 || c->dev >= ATTR_DEVS) return set_err(GK_ERR_ARG, "device id %d out of range", c->dev);
    if (p.r2e > RW || p.lds < LX * RES_PC_NT * (int)sizeof(double2))
        return set_err(GK_ERR_STATE, "column-cache plan (%d chunks, %d B LDS) does not fit k_mgs_wpc<%d,%d,%d>", p.r2e,
                       p.lds, RW, RX, LX);
    if (p.lds > 0 && attr[c->dev].load() < p.lds) {
        HIPCHK(hipFuncSetAttribute(
            reinterpret_cast<const void *>(&gk::k_mgs_wpc<RW, RX, LX, MODE, WBT, RES_PC_TOUCH, RES_PC_NT>),
            hipFuncAttributeMaxDynamicSharedMemorySize, p.lds));
        attr[c->dev] = p.lds;
    }
    gk::k_mgs_wpc<RW, RX, LX, MODE, WBT, RES_PC_TOUCH, RES_PC_NT><<<p.G, RES_PC_NT, p.lds, c->st>>>(a);
    LAUNCHCHK();
    return GK_OK;
}

template <int MODE>
int launch_wpc_m(gk_ctx *c, const ResPlan &p, const gk::ResArgs &a) {
    if constexpr (RES_PCS) {
        if (p.pcs) return launch_wpc_k<RES_PCS_RW, RES_PCS_RX, RES_PCS_LX, MODE>(c, p, a);
    }
    return launch_wpc_k<RES_PC_RW, MODE == gk::RES_MGS ? RES_PC_RX_MGS : RES_PC_RX, RES_PC_LX, MODE>(c, p, a);
}

int launch_res(gk_ctx *c, const ResPlan &p, const gk::ResArgs &a) {
    if (p.bvar >= 0) {
        if (a.mode != gk::RES_MGS) return set_err(GK_ERR_STATE, "the blocked step is the MGS-R step's only");
        const int e = gk::blk_launch(p.bvar, p.blk, a, p.G, p.lds, c->dev, c->st);
        if (e != 0)
            return set_err(GK_ERR_HIP, "k_mgs_blk (S=%d, variant %d): %s", p.blk, p.bvar,
                           hipGetErrorString(static_cast<hipError_t>(e)));
        return GK_OK;
    }
    if (p.wo) return launch_wres(c, p, a);
    if (p.pc) {
        switch (a.mode) {
            case gk::RES_HH_UP: return launch_wpc_m<gk::RES_HH_UP>(c, p, a);
            case gk::RES_HH_DOWN: return launch_wpc_m<gk::RES_HH_DOWN>(c, p, a);
            default: return launch_wpc_m<gk::RES_MGS>(c, p, a);
        }
    }
#define GK_RES_CASE(R, L, PFV, CWV)                                                                 \
    if (p.r2 == R && p.l2 == L && p.pf == PFV && p.cw == CWV)                                      \
        return p.nt ? launch_res_t<R, L, PFV, true, CWV>(c, p, a) : launch_res_t<R, L, PFV, false, CWV>(c, p, a);
    GK_RES_CASE(2, 0, true, true)
    GK_RES_CASE(4, 0, true, true)
    GK_RES_CASE(8, 0, true, true)
    GK_RES_CASE(RES_R2_BIG, 0, false, false)
    GK_RES_CASE(RES_R2_BIG, RES_L2, false, false)
#undef GK_RES_CASE
    return set_err(GK_ERR_ARG, "no resident variant for r2=%d l2=%d", p.r2, p.l2);
}

// One resident launch (gk::ResArgs::mode):
//  RES_MGS: the MGS cascade of step j + norm + scale; pin/npin = the
//    (all-reduced) partial slab of the first dot <w, V(:,1)>; H column to hs/hcopy.
//  RES_HH_UP: w = P_j..P_1 w (pin = <w, P_1>); hs[0] = ||w(j+1:n)||^2.
//  RES_HH_DOWN: w = P_1..P_j w (no pin).
//  flags (w-only variant, p.wo): RESF_CLOSE_HH -- RES_HH_UP also makes P(:,j+1) and
//    writes w(1:j+1) to c->hb (one more exchange); RESF_UNIT_INIT -- RES_HH_DOWN builds
//    its unit input e_{unit_g} itself.
enum { RESF_CLOSE_HH = 1, RESF_UNIT_INIT = 2, RESF_PIN_LOCAL = 4 };
int res_step(gk_ctx *c, int j, const ResPlan &p, const double *pin, int npin, double *hs, double *hcopy,
             int mode = gk::RES_MGS, double *w = nullptr, i64 unit_g = -1, int flags = 0) {
    ProfScope ps(c, GK_KID_RES);
    const bool close = (flags & RESF_CLOSE_HH) && mode == gk::RES_HH_UP;
    if ((flags & ~RESF_PIN_LOCAL) != 0 && !p.wo)
        return set_err(GK_ERR_STATE, "resident flags %d need the w-only variant", flags);
    const bool pin_local = (flags & RESF_PIN_LOCAL) && mode != gk::RES_HH_DOWN && c->xs_on && c->nranks > 1;
    // exchanges of the launch
    const int np = (mode == gk::RES_MGS ? (p.bvar >= 0 ? gk::blk_exchanges(j, p.blk) : 2 * j) : j) + (close ? 1 : 0);
    if (c->res_tag > 0xF0000000u) {  // tags must never repeat within the granule region's lifetime
        HIPCHK(hipMemsetAsync(c->res_gath, 0, sizeof(gk::u64) * gk::RES_GATH_ALL, c->st));
        c->res_tag = 1;
    }
    gk::ResArgs a{};
    a.w = w != nullptr ? w : c->w;
    a.mode = mode;
    a.coef = mode == gk::RES_MGS ? 1.0 : 2.0;
    a.tail0 = mode == gk::RES_HH_UP ? (i64)j - c->g0 : 0;
    a.V = c->V;
    a.vout = c->V + (i64)j * c->ld;
    a.ld = c->ld;
    a.pin = pin;
    a.npin = npin;
    a.hs = hs;
    a.hcopy = hcopy;
    a.gath = c->res_gath;
    a.gm = c->res_gm;
    a.j = j;
    a.n = c->nloc;
    a.nres2 = p.nres2;
    a.r2e = p.r2e;
    a.l2e = p.l2e;
    a.unit_known = mode == gk::RES_HH_DOWN && unit_g >= 0;
    a.unit_e = (a.unit_known && unit_g >= c->g0 && unit_g < c->g0 + c->nloc) ? unit_g - c->g0 : -1;
    a.unit_init = a.unit_known && (flags & RESF_UNIT_INIT) ? 1 : 0;
    a.close_hh = close ? 1 : 0;
    a.hb = c->hb;
    a.tag0 = c->res_tag;
    c->res_tag += (unsigned)np;
    a.timeout = (gk::u64)c->res_timeout_ms * (gk::u64)c->xs_tick_per_ms;
    a.err = c->res_err_dev;
    a.stamps = c->res_split ? c->res_stamps : nullptr;
    if (c->res_trace != nullptr && j == c->res_trace_j && mode == c->res_trace_mode) {
        a.trace = c->res_trace;
        c->res_trace_g = p.G;
        c->res_trace_np = np;
    }
    // auto: on -- A/B at 2896^2 (k_mgs_res<12, 18> NT, profiles/r04/ab_qdef_2896_r04a.jsonl): 19.98 /
    // 19.90 -> 18.82 / 18.84 us per projection
    a.qdef = c->tune_res_qdef != 0 ? 1 : 0;
    a.nranks = 1;
    if (c->xs_on && c->nranks > 1) {
        a.err = c->xs_err_dev;
        a.timeout = std::max(a.timeout, c->xs_timeout);
        a.peers = c->xs_peers;
        a.nranks = c->nranks;
        a.rank = c->rank;
        a.pin_local = pin_local ? 1 : 0;  // the first dot's rank hop takes the launch's first number
        a.xseq0 = c->xs_seq + (pin_local ? 1u : 0u);
        c->xs_seq += (unsigned)np + (pin_local ? 1u : 0u);
    }
    return launch_res(c, p, a);
}


int d2h_sync(gk_ctx *c, double *host, const double *dev, int count) {
    HIPCHK(hipMemcpyAsync(c->hcol_host, dev, sizeof(double) * count, hipMemcpyDeviceToHost, c->st));
    CHK(sync_st(c));
    if (c->prof) CHK(prof_harvest(c));
    std::memcpy(host, c->hcol_host, sizeof(double) * count);
    return GK_OK;
}

int precond_sweeps(gk_ctx *c, double *out, int acc, const double *vdot, double *part);

// out = M^-1 (A v)  or  out = M^-1 (b - A v) (resid); the LAST sweep carries
// the fused reduction `acc` (dot with vdot, or norm) into slab `part`.
// Reference: gmres_mgsr.f90:336-337 (step), :314-320 (cycle start).
int op_precond_sten(gk_ctx *c, const double *v, double *out, int acc, const double *vdot, double *part,
                    bool *done);
int op_precond(gk_ctx *c, const double *v, double *out, bool resid, int acc, const double *vdot,
               double *part) {
    if (!resid) {
        bool done = false;
        CHK(op_precond_sten(c, v, out, acc, vdot, part, &done));
        if (done) return GK_OK;
    }
    CHK(halo(c, v));
    gk::StArgs a{};
    if (c->pkind == GK_PREC_IDENTITY) {
        a.x = v;
        a.in1 = c->b;
        a.y = out;
        a.vdot = vdot;
        a.part = part;
        return stencil(c, resid ? gk::OP_RESID : gk::OP_PLAIN, acc, a);
    }
    // z = A v   (or b - A v)
    a.x = v;
    a.in1 = c->b;
    a.y = c->z;
    CHK(stencil(c, resid ? gk::OP_RESID : gk::OP_PLAIN, gk::ACC_NONE, a));
    return precond_sweeps(c, out, acc, vdot, part);
}

// The Arnoldi step's out = M^-1 (A v) with Chebyshev(k <= 8) as ONE pass whose
// stage 0 forms z = A v itself: no stencil launch, no z vector (the pass reads
// v; on slabs v brings k + 1 deep-halo lines).  *done = false: not applicable
// (the caller takes the stencil + pass route).
int cheb_fused_ok(gk_ctx *c, bool *ok);
int cheb_coefs(gk_ctx *c, double *c1, double *c2, double *theta);
int cheb_fused(gk_ctx *c, double *out, int acc, const double *vdot, double *part, const double *c1,
               const double *c2, double theta, const double *sten_v);
int op_precond_sten(gk_ctx *c, const double *v, double *out, int acc, const double *vdot, double *part,
                    bool *done) {
    *done = false;
    if (c->pkind != GK_PREC_CHEB || acc != gk::ACC_DOT || !c->tune_cheb_sten || c->pdeg > gk::CF_LMAX ||
        c->N < gk::CF_PTS)
        return GK_OK;
    bool fused = false;
    CHK(cheb_fused_ok(c, &fused));
    if (!fused || (collective(c) && c->nranks > 1 && c->min_lines < c->pdeg + 1)) return GK_OK;
    double c1[2 * gk::CF_LMAX], c2[2 * gk::CF_LMAX], theta;
    CHK(cheb_coefs(c, c1, c2, &theta));
    CHK(cheb_fused(c, out, acc, vdot, part, c1, c2, theta, v));
    *done = true;
    return GK_OK;
}

// One temporal-blocked pass (gk_cheb.hip), tiles sized by the largest slab so
// every rank writes the same number of partials (the all-reduced slab has one
// length on all ranks).
template <bool FIRST, bool LAST>
int launch_cf(gk_ctx *c, int L, int acc, gk::CFArgs &a, i64 *np, bool sten = false) {
    gk::CFLaunch q{};
    q.L = L;
    q.sten = sten;
    q.first = FIRST;
    q.last = LAST;
    q.acc = acc;
    q.lines = (c->nranks > 1 && c->max_lines > c->nlines) ? c->max_lines : c->nlines;
    q.cus = c->res_cus > 0 ? c->res_cus : 256;
    q.dev = c->dev;
    q.st = c->st;
    const int e = gk::cheb_launch(q, a, np);
    if (e == gk::GK_CF_ESLOT) return set_err(GK_ERR_ARG, "Chebyshev pass grid exceeds a reduction slot");
    if (e == gk::GK_CF_ESTEN) return set_err(GK_ERR_ARG, "fused-stencil Chebyshev pass outside its variants");
    if (e == gk::GK_CF_ESPILL)
        return set_err(GK_ERR_HIP, "Chebyshev pass (L = %d) was built with a register spill to scratch; refused", L);
    if (e != 0) return set_err(GK_ERR_HIP, "Chebyshev pass launch: %s", hipGetErrorString((hipError_t)e));
    return GK_OK;
}

// Chebyshev(k <= 16) as one or two temporal-blocked passes (gk_cheb.hip):
// sweeps 1..min(k, 8) in the first, the rest in the second.
int cheb_fused(gk_ctx *c, double *out, int acc, const double *vdot, double *part, const double *c1,
               const double *c2, double theta, const double *sten_v) {
    ProfScope ps(c, GK_KID_PREC);
    const int k = c->pdeg;
    const int g1 = std::min(k, gk::CF_LMAX), g2 = k - g1;
    const bool sten = sten_v != nullptr;  // one pass (k <= 8) taking v, stage 0 = the stencil
    // On slabs every input of a pass brings L lines of each neighbour (deep halo).
    const bool slabs = collective(c) && c->nranks > 1;
    const bool has_lo = slabs && c->rank > 0, has_hi = slabs && c->rank < c->nranks - 1;
    auto dlo = [&](int v) { return c->dh + (i64)(2 * v) * gk::CF_HMAX * c->N; };
    auto dhi = [&](int v) { return c->dh + (i64)(2 * v + 1) * gk::CF_HMAX * c->N; };
    auto deep = [&](gk::CFArgs &x, int v, const double *vec, int L) -> int {
        if (slabs) CHK(halo_lines(c, vec, L, dlo(v), dhi(v)));
        x.lo[v] = has_lo ? dlo(v) : nullptr;
        x.hi[v] = has_hi ? dhi(v) : nullptr;
        return GK_OK;
    };
    gk::CFArgs a{};
    a.N = c->N;
    a.nlines = c->nlines;
    a.theta = theta;
    a.din = sten ? sten_v : c->z;
    a.vdot = vdot;
    a.part = part;
    CHK(deep(a, 0, a.din, g1 + (sten ? 1 : 0)));
    for (int l = 0; l < g1; ++l) {
        a.c1[l] = c1[l];
        a.c2[l] = c2[l];
    }
    i64 np = 0;
    if (g2 == 0) {
        a.out = out;
        CHK((launch_cf<true, true>(c, g1, acc, a, &np, sten)));
        if (acc != gk::ACC_NONE) c->last_np = (int)np;
        return GK_OK;
    }
    a.dout = c->dA;
    a.rout = c->aux;
    a.zout = c->dB;
    CHK((launch_cf<true, false>(c, g1, gk::ACC_NONE, a, nullptr)));
    gk::CFArgs b{};
    b.N = c->N;
    b.nlines = c->nlines;
    b.din = c->dA;
    b.rin = c->aux;
    b.zin = c->dB;
    CHK(deep(b, 0, c->dA, g2));
    CHK(deep(b, 1, c->aux, g2));
    CHK(deep(b, 2, c->dB, g2));
    b.out = out;
    b.vdot = vdot;
    b.part = part;
    for (int l = 0; l < g2; ++l) {
        b.c1[l] = c1[g1 + l];
        b.c2[l] = c2[g1 + l];
    }
    CHK((launch_cf<false, true>(c, g2, acc, b, &np)));
    if (acc != gk::ACC_NONE) c->last_np = (int)np;
    return GK_OK;
}

// The smallest slab of any rank, gathered once per communicator (collective:
// every rank reaches it at the same point, the first Chebyshev application):
// each rank contributes its nlines at its own position of a short vector that
// is all-reduced by sum.  The decomposition may be any set of consecutive
// slabs (gk_create / gk_comm_init take any line0, nlines), not only
// slab_partition's.
int ensure_min_lines(gk_ctx *c) {
    if (c->min_lines > 0) return GK_OK;
    if (!collective(c) || c->nranks == 1) {
        c->min_lines = c->nlines;
        return GK_OK;
    }
    std::vector<double> v(c->nranks, 0.0);
    v[c->rank] = c->nlines;
    double *d = slot(c, 3);
    HIPCHK(hipMemcpyAsync(d, v.data(), sizeof(double) * c->nranks, hipMemcpyHostToDevice, c->st));
    CHK(allreduce(c, d, c->nranks, true));
    HIPCHK(hipMemcpyAsync(v.data(), d, sizeof(double) * c->nranks, hipMemcpyDeviceToHost, c->st));
    CHK(sync_st(c));
    int mn = c->nlines;
    for (double x : v) mn = std::min(mn, (int)x);
    c->min_lines = mn;
    return GK_OK;
}

// Temporal-blocked Chebyshev passes: even N (two points per lane), k <= 16,
// slabs below 2 GiB per vector, and on slabs every rank holding at least the
// pass's L lines (the deep halo comes from the immediate neighbour only).  The
// same answer on every rank.
int cheb_fused_ok(gk_ctx *c, bool *ok) {
    *ok = false;
    if (!c->tune_cheb_fused || c->N % 2 != 0 || c->pdeg > 2 * gk::CF_LMAX) return GK_OK;
    // the pass addresses slab vectors through 32-bit buffer offsets
    if ((i64)c->N * std::max(c->nlines, c->max_lines) * 8 >= (1LL << 31)) return GK_OK;
    if (!collective(c) || c->nranks == 1) {
        *ok = true;
        return GK_OK;
    }
    CHK(ensure_min_lines(c));
    *ok = c->min_lines >= std::min(c->pdeg, gk::CF_LMAX);
    return GK_OK;
}

// Chebyshev(k) coefficients of the sweeps (the per-sweep kernels' recurrence).
int cheb_coefs(gk_ctx *c, double *c1, double *c2, double *theta) {
    *theta = (c->p0 + c->p1) / 2.0;
    const double delta = std::fabs(c->p1 - c->p0) / 2.0;
    const double sigma = *theta / delta;
    double rho0 = delta / *theta;
    for (int it = 0; it < c->pdeg; ++it) {
        const double rho1 = 1.0 / (2.0 * sigma - rho0);
        c1[it] = rho1 * rho0;
        c2[it] = 2.0 * rho1 / delta;
        rho0 = rho1;
    }
    return GK_OK;
}

// out = M^-1 z for z already in c->z (cbpr2 or Chebyshev sweeps).
int precond_sweeps(gk_ctx *c, double *out, int acc, const double *vdot, double *part) {
    bool fused = false;
    if (c->pkind == GK_PREC_CHEB) CHK(cheb_fused_ok(c, &fused));
    if (!fused) CHK(halo(c, c->z));  // the fused passes bring their own deep halos
    if (c->pkind == GK_PREC_CBPR2) {
        // cbpr2 coefficients exactly as chebyshev.f90:19-25
        const double em = c->p0, eM = c->p1;
        const double cc = (eM - em) / 2.0;
        const double d = (eM + em) / 2.0;
        double alpha = 1.0 / d;
        double beta = cc * alpha / 2.0;
        beta = beta * beta;
        alpha = 1.0 / (d - beta);
        gk::StArgs b2{};
        b2.x = c->z;
        b2.y = out;
        b2.vdot = vdot;
        b2.part = part;
        b2.s1 = d;
        b2.s2 = alpha;
        return stencil(c, gk::OP_CBPR2, acc, b2);
    }
    // Chebyshev(k): k sweeps, each one stencil on d_k fused with the three
    // vector updates (res, d, z); the first sweep builds d_0 = r/theta on load.
    const double theta = (c->p0 + c->p1) / 2.0;
    const double delta = std::fabs(c->p1 - c->p0) / 2.0;
    const double sigma = theta / delta;
    double rho0 = delta / theta;
    if (fused) {
        double c1[2 * gk::CF_LMAX], c2[2 * gk::CF_LMAX], th;
        CHK(cheb_coefs(c, c1, c2, &th));
        return cheb_fused(c, out, acc, vdot, part, c1, c2, th, nullptr);
    }
    double *dcur = c->dA, *dnext = c->dB;
    for (int it = 0; it < c->pdeg; ++it) {
        const double rho1 = 1.0 / (2.0 * sigma - rho0);
        const double c1 = rho1 * rho0, c2 = 2.0 * rho1 / delta;
        const bool last = (it == c->pdeg - 1);
        gk::StArgs s{};
        s.y = out;
        s.s2 = c1;
        s.s3 = c2;
        s.vdot = vdot;
        s.part = part;
        if (it == 0) {
            s.x = c->z;
            s.s1 = theta;
            s.o_res = last ? nullptr : c->aux;
            s.o_d = last ? nullptr : dcur;
            CHK(stencil(c, gk::OP_CHEB_FIRST, last ? acc : gk::ACC_NONE, s));
        } else {
            CHK(halo(c, dcur));
            s.x = dcur;
            s.in1 = c->aux;
            s.in2 = out;
            s.o_res = last ? nullptr : c->aux;
            s.o_d = last ? nullptr : dnext;
            CHK(stencil(c, gk::OP_CHEB_ITER, last ? acc : gk::ACC_NONE, s));
            std::swap(dcur, dnext);
        }
        rho0 = rho1;
    }
    return GK_OK;
}

int owner_of(gk_ctx *c, i64 gidx) {
    // ranks own consecutive slabs; rank r owns [g0_r, g0_r + nloc_r). Only the
    // HH path needs this and only for gidx <= m, which lives on the rank whose
    // slab starts at line 0 when N >= m+1 (checked at cycle start).
    (void)gidx;
    return 0;
}

int check_ctx(gk_ctx *c) {
    if (c == nullptr) return set_err(GK_ERR_ARG, "null context");
    if (c->broken)
        return set_err(GK_ERR_STATE, "context broken by an earlier watchdog timeout (work never completed on its "
                                     "stream): destroy it");
    if (c->nranks > 1 && !c->comm_ok) return set_err(GK_ERR_STATE, "communicator not initialised");
    return GK_OK;
}

// The orthogonality diagnostics in the reference's summation order (one running
// sum per dot, gk::seq_dot) unless tuned off; a running sum cannot cross a slab
// boundary without serialising the ranks, so N ranks use the tree (k_gram).
bool verr_ref_order(const gk_ctx *c) { return c->tune_verr_order != 0 && c->nranks == 1; }

int ensure_gram(gk_ctx *c, int ncols) {
    if (ncols > gk::GCMAX) return set_err(GK_ERR_ARG, "v_err needs <= %d columns", gk::GCMAX);
    if (c->gram_slab == nullptr) {
        c->gram_nblk = 512;
        const int maxpairs = gk::GCMAX * (gk::GCMAX + 1) / 2;
        HIPCHK(hipMalloc(&c->gram_slab, sizeof(double) * (size_t)c->gram_nblk * maxpairs));
        HIPCHK(hipMalloc(&c->gram_out, sizeof(double) * maxpairs));
        HIPCHK(hipMalloc(&c->gram_pairs, sizeof(short2) * maxpairs));
    }
    return GK_OK;
}

// G (host, c x c symmetric, column-major) of the first c columns of base.
int gram(gk_ctx *c, const double *base, int ncols, std::vector<double> &G) {
    CHK(ensure_gram(c, ncols));
    std::vector<short2> pr;
    for (int bb = 0; bb < ncols; ++bb)
        for (int aa = 0; aa <= bb; ++aa) pr.push_back(make_short2((short)aa, (short)bb));
    const int np = (int)pr.size();
    HIPCHK(hipMemcpyAsync(c->gram_pairs, pr.data(), sizeof(short2) * np, hipMemcpyHostToDevice, c->st));
    if (verr_ref_order(c)) {  // one running sum per pair, k in order (the reference's dot_product)
        ProfScope ps(c, GK_KID_OTHER);
        gk::k_seqdot_pairs<<<(np + 63) / 64, 64, 0, c->st>>>(base, c->ld, c->nloc, c->gram_pairs, np, c->gram_out);
        LAUNCHCHK();
    } else {
        ProfScope ps(c, GK_KID_OTHER);
        gk::k_gram<<<c->gram_nblk, gk::TPB, 0, c->st>>>(base, c->ld, ncols, c->nloc, c->gram_pairs, np,
                                                        c->gram_slab);
        LAUNCHCHK();
        gk::k_gram_reduce<<<(np + gk::TPB - 1) / gk::TPB, gk::TPB, 0, c->st>>>(c->gram_slab, c->gram_nblk,
                                                                            np, c->gram_out);
        LAUNCHCHK();
        CHK(allreduce(c, c->gram_out, np, true));
    }
    std::vector<double> flat(np);
    HIPCHK(hipMemcpyAsync(flat.data(), c->gram_out, sizeof(double) * np, hipMemcpyDeviceToHost, c->st));
    CHK(sync_st(c));
    if (c->prof) CHK(prof_harvest(c));
    G.assign((size_t)ncols * ncols, 0.0);
    for (int p = 0; p < np; ++p) {
        G[(size_t)pr[p].y * ncols + pr[p].x] = flat[p];
        G[(size_t)pr[p].x * ncols + pr[p].y] = flat[p];
    }
    return GK_OK;
}

// v <- P_1 .. P_k v  (apply reflections k..1; hh_step :269-283, update :361-373,
// calculate_verr :581-585).  The chain's first launch is a pure dot.
// unit_g >= 0: v is the unit vector e at global index unit_g (gk_hh_step's v_j,
// calculate_verr's columns), so the chain's leading dot <e, P_k> is the single
// element P_k(unit_g) -- exactly what the full dot sums to -- and the resident
// launch skips that pass.
int reflect_chain_down(gk_ctx *c, double *v, int k, i64 unit_g = -1, int flags = 0) {
    double *P = c->V;
    ResPlan rp;
    if (res_plan(c, rp, true))
        return res_step(c, k, rp, nullptr, 0, nullptr, nullptr, gk::RES_HH_DOWN, v, unit_g, flags);
    if (flags != 0) return set_err(GK_ERR_STATE, "resident chain flags without a resident plan");
    int s0 = 0, s1 = 1;
    CHK(proj(c, gk::PJ_DOT, v, nullptr, P + (i64)(k - 1) * c->ld, nullptr, 0, slot(c, s0), nullptr, 2.0));
    int np = c->np_pj;
    for (int i = k; i >= 1; --i) {
        CHK(allreduce(c, slot(c, s0), np));
        const double *va = P + (i64)(i - 1) * c->ld;
        if (i > 1) {
            CHK(proj(c, gk::PJ_AXPY_DOT, v, va, P + (i64)(i - 2) * c->ld, slot(c, s0), np, slot(c, s1),
                     nullptr, 2.0));
            std::swap(s0, s1);
        } else {
            CHK(proj(c, gk::PJ_AXPY, v, va, nullptr, slot(c, s0), np, nullptr, nullptr, 2.0));
        }
    }
    return GK_OK;
}

// The launch path's MGS-R cascade of step j after the operator launch left the
// first dot's partial slab (np partials) in slot 0: two passes of j projections
// (AXPY_i fused with dot_{i+1}), each dot all-reduced, then h = ||w|| and
// V(:,j+1) = w / h with H(1:j+1, j) published to mapped host memory.
// gmres_mgsr.f90:341-363, :384.
int mgs_chain(gk_ctx *c, int j, int np) {
    const i64 ld = c->ld;
    double *V = c->V;
    const int m2 = c->m + 2;
    double *hs = c->hall + (i64)(j - 1) * m2;
    int s0 = 0, s1 = 1;
    const int np_total = 2 * j;
    for (int p = 0; p < np_total; ++p) {
        const int i = p % j;
        CHK(allreduce(c, slot(c, s0), np));
        const double *va = V + (i64)i * ld;
        const int first_pass = p < j;
        if (p + 1 < np_total) {
            const double *vb = V + (i64)((p + 1) % j) * ld;
            CHK(proj(c, gk::PJ_AXPY_DOT, c->w, va, vb, slot(c, s0), np, slot(c, s1), hs + i, 1.0, 0, first_pass));
        } else {
            CHK(proj(c, gk::PJ_AXPY_NORM, c->w, va, nullptr, slot(c, s0), np, slot(c, s1), hs + i, 1.0, 0,
                     first_pass));
        }
        np = c->np_pj;
        std::swap(s0, s1);
    }
    CHK(allreduce(c, slot(c, s0), np));
    return scale(c, V + (i64)j * ld, c->w, slot(c, s0), np, hs + j, c->hallh_dev + (i64)(j - 1) * m2, hs, j);
}

// Capture mgs_chain(j) once as a graph (its kernel arguments and communicator
// calls depend only on j, np and the context's fixed buffers).  A capture that
// fails switches graphs off for this context; one rank then runs the step call by
// call.  With an RCCL communicator the failure is an error instead: the discarded
// graph may already hold some of the step's ncclAllReduce calls, and whether RCCL's
// per-communicator operation counters stay matched when one rank runs eagerly while
// its peers replay is not pinned -- the caller reruns with GK_TUNE_GRAPH 0 on every
// rank.  (GK_DEBUG_CAPTURE_FAIL=1 makes every capture fail after it ends, for tests.)
int capture_step(gk_ctx *c, int j, int np) {
    HIPCHK(hipStreamBeginCapture(c->st, hipStreamCaptureModeThreadLocal));
    c->capturing = true;
    c->graph_seq0 = c->xs_seq;
    const int rc = mgs_chain(c, j, np);
    c->capturing = false;
    const unsigned nxs = c->xs_seq - c->graph_seq0;  // nothing ran: the numbers are reused by the replay
    c->xs_seq = c->graph_seq0;
    if ((int)c->gxs.size() < c->m + 1) c->gxs.resize(c->m + 1, 0);
    c->gxs[j] = nxs;
    hipGraph_t g = nullptr;
    const hipError_t e = hipStreamEndCapture(c->st, &g);
    hipGraphExec_t ge = nullptr;
    hipError_t e2 = hipErrorUnknown;
    if (rc == GK_OK && e == hipSuccess && g != nullptr) e2 = hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    if (g != nullptr) (void)hipGraphDestroy(g);
    const char *dbg = std::getenv("GK_DEBUG_CAPTURE_FAIL");
    const bool forced = dbg != nullptr && dbg[0] == '1';
    if (rc != GK_OK || e != hipSuccess || e2 != hipSuccess || forced) {
        const std::string why = rc != GK_OK ? g_err
                                : forced   ? std::string("GK_DEBUG_CAPTURE_FAIL")
                                           : hipGetErrorString(e != hipSuccess ? e : e2);
        (void)hipGetLastError();
        if (ge != nullptr) (void)hipGraphExecDestroy(ge);
        c->tune_graph = 0;
        graph_reset(c);
        if (c->comm != nullptr && !c->xs_on && c->lg == nullptr)  // the step's all-reduces are RCCL calls
            return set_err(GK_ERR_COMM,
                           "capture of launch-path step %d failed on an RCCL rank (%s): rerun with GK_TUNE_GRAPH 0 "
                           "on every rank (one rank running the step eagerly while its peers replay graphs is not "
                           "supported)", j, why.c_str());
        set_err(GK_OK, "launch-path step graphs off for this context: capture of step %d failed (%s)", j,
                why.c_str());
        return GK_OK;
    }
    c->gstep[j] = ge;
    return GK_OK;
}

}  // namespace

// ======================================================================= API

extern "C" {

const char *gk_last_error(void) { return g_err.c_str(); }
int gk_version(void) { return 1; }

int gk_runtime_info(int *hip_runtime, int *hip_driver, int *rccl, char *hip_path, char *rccl_path, int len) {
    if (hip_runtime == nullptr || hip_driver == nullptr || rccl == nullptr) return set_err(GK_ERR_ARG, "null argument");
    *hip_runtime = *hip_driver = *rccl = 0;
    HIPCHK(hipRuntimeGetVersion(hip_runtime));
    HIPCHK(hipDriverGetVersion(hip_driver));
    NCCLCHK(ncclGetVersion(rccl));
    auto path_of = [&](const void *sym, char *out) {
        if (out == nullptr || len <= 0) return;
        Dl_info di{};
        const char *p = (dladdr(sym, &di) != 0 && di.dli_fname != nullptr) ? di.dli_fname : "";
        std::snprintf(out, (size_t)len, "%s", p);
    };
    path_of(reinterpret_cast<const void *>(&hipRuntimeGetVersion), hip_path);
    path_of(reinterpret_cast<const void *>(&ncclGetVersion), rccl_path);
    return GK_OK;
}

int gk_create(int device, int nside, int line0, int nlines, int m, gk_ctx **out) {
    if (out == nullptr) return set_err(GK_ERR_ARG, "null out");
    *out = nullptr;
    if (nside < 2 || nlines < 1 || line0 < 0 || line0 + nlines > nside || m < 1 || m > 4096)
        return set_err(GK_ERR_ARG, "bad shape N=%d line0=%d nlines=%d m=%d", nside, line0, nlines, m);
    HIPCHK(hipSetDevice(device));
    gk_ctx *c = new gk_ctx();
    c->dev = device;
    c->N = nside;
    c->line0 = line0;
    c->nlines = nlines;
    c->m = m;
    c->nloc = (i64)nside * nlines;
    c->g0 = (i64)nside * line0;
    c->ld = round_up(c->nloc, 32);  // 256-byte aligned columns
    c->max_lines = nlines;
    set_geometry(c);
    auto fail = [&](int code) {
        gk_destroy(c);
        return code;
    };
    if (hipStreamCreateWithFlags(&c->st, hipStreamNonBlocking) != hipSuccess)
        return fail(set_err(GK_ERR_HIP, "stream create failed"));
    const size_t vb = sizeof(double) * (size_t)c->ld;
    if (hipMalloc(&c->V, vb * (m + 1)) != hipSuccess)
        return fail(set_err(GK_ERR_NOMEM, "cannot allocate V: %.2f GB", vb * (m + 1) / 1e9));
    double **vecs[] = {&c->w, &c->z, &c->aux, &c->dA, &c->dB, &c->x, &c->b, &c->vj};
    for (double **p : vecs)
        if (hipMalloc(p, vb) != hipSuccess) return fail(set_err(GK_ERR_NOMEM, "cannot allocate work vectors"));
    if (hipMalloc(&c->hlo, sizeof(double) * nside) != hipSuccess ||
        hipMalloc(&c->hhi, sizeof(double) * nside) != hipSuccess ||
        hipMalloc(&c->dh, sizeof(double) * 6 * gk::CF_HMAX * (size_t)nside) != hipSuccess ||
        hipMalloc(&c->zline, sizeof(double) * (size_t)nside) != hipSuccess ||
        hipMemsetAsync(c->zline, 0, sizeof(double) * (size_t)nside, c->st) != hipSuccess ||
        hipMalloc(&c->red, sizeof(double) * NSLOT * gk::NPMAX) != hipSuccess ||
        hipMalloc(&c->hcol, sizeof(double) * (m + 2)) != hipSuccess ||
        hipMalloc(&c->ydev, sizeof(double) * (m + 1)) != hipSuccess ||
        hipMalloc(&c->hb, sizeof(double) * (m + 2)) != hipSuccess ||
        hipMalloc(&c->scal, sizeof(double) * 8) != hipSuccess)
        return fail(set_err(GK_ERR_NOMEM, "cannot allocate small buffers"));
    if (hipHostMalloc(&c->hcol_host, sizeof(double) * (m + 2 + gk::GCMAX)) != hipSuccess)
        return fail(set_err(GK_ERR_NOMEM, "cannot allocate pinned buffer"));
    if (hipMalloc(&c->hall, sizeof(double) * (size_t)(m + 2) * (m + 1)) != hipSuccess ||
        hipHostMalloc(&c->hallh, sizeof(double) * (size_t)(m + 2) * (m + 1), hipHostMallocMapped) != hipSuccess ||
        hipHostGetDevicePointer((void **)&c->hallh_dev, c->hallh, 0) != hipSuccess)
        return fail(set_err(GK_ERR_NOMEM, "cannot allocate the Hessenberg mirrors"));
    if (hipMalloc(&c->res_gath, sizeof(gk::u64) * gk::RES_GATH_ALL) != hipSuccess ||
        hipMalloc(&c->res_gm, sizeof(double) * (size_t)(m + 1 + gk::RES_SMAX) * gk::RES_SMAX) != hipSuccess ||
        hipHostMalloc((void **)&c->res_err, sizeof(int), hipHostMallocMapped) != hipSuccess ||
        hipHostGetDevicePointer((void **)&c->res_err_dev, c->res_err, 0) != hipSuccess ||
        hipMemsetAsync(c->res_gm, 0, sizeof(double) * (size_t)(m + 1 + gk::RES_SMAX) * gk::RES_SMAX, c->st) != hipSuccess ||
        hipMemsetAsync(c->res_gath, 0, sizeof(gk::u64) * gk::RES_GATH_ALL, c->st) != hipSuccess)
        return fail(set_err(GK_ERR_NOMEM, "cannot allocate the resident-step exchange area"));
    *c->res_err = 0;
    {
        int cus = 0, khz = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess) c->res_cus = cus;
        if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device) == hipSuccess && khz > 0)
            c->xs_tick_per_ms = khz;
    }
    c->ev_step.assign(m + 1, nullptr);
    for (int k = 0; k <= m; ++k)
        if (hipEventCreateWithFlags(&c->ev_step[k], hipEventDisableTiming) != hipSuccess)
            return fail(set_err(GK_ERR_HIP, "event create failed"));
    if (hipMemsetAsync(c->x, 0, vb, c->st) != hipSuccess || hipMemsetAsync(c->b, 0, vb, c->st) != hipSuccess ||
        hipMemsetAsync(c->V, 0, vb * (m + 1), c->st) != hipSuccess ||
        hipMemsetAsync(c->red, 0, sizeof(double) * NSLOT * gk::NPMAX, c->st) != hipSuccess)
        return fail(set_err(GK_ERR_HIP, "memset failed"));
    c->ev0.resize(PROF_POOL);
    c->ev1.resize(PROF_POOL);
    c->evk.resize(PROF_POOL);
    for (int k = 0; k < PROF_POOL; ++k) {
        if (hipEventCreate(&c->ev0[k]) != hipSuccess || hipEventCreate(&c->ev1[k]) != hipSuccess)
            return fail(set_err(GK_ERR_HIP, "event create failed"));
    }
    if (hipStreamSynchronize(c->st) != hipSuccess) return fail(set_err(GK_ERR_HIP, "sync failed"));
    *out = c;
    return GK_OK;
}

int gk_destroy(gk_ctx *c) {
    if (c == nullptr) return GK_OK;
    (void)hipSetDevice(c->dev);
    if (c->broken && c->st) {
        // a broken context's stream may never drain: wait a bounded time, and leak the
        // context (rather than free memory its kernels may still touch) if it does not
        if (spin_until(c, query_stream, c->st, "destroy of a broken context") != GK_OK)
            return set_err(GK_ERR_COMM, "gk_destroy: the broken context's stream did not drain; its memory is kept");
    }
    if (c->st) (void)hipStreamSynchronize(c->st);
    graph_reset(c);
    if (c->comm) ncclCommDestroy(c->comm);
    if (c->lev_a) (void)hipEventDestroy(c->lev_a);
    if (c->lev_b) (void)hipEventDestroy(c->lev_b);
    if (c->lscratch) (void)hipFree(c->lscratch);
    for (void *p : c->xs_mapped) (void)hipIpcCloseMemHandle(p);
    if (c->xs_buf) (void)hipFree(c->xs_buf);
    if (c->xs_seqdev) (void)hipFree(c->xs_seqdev);
    if (c->xs_err) (void)hipHostFree(c->xs_err);
    if (c->res_gath) (void)hipFree(c->res_gath);
    if (c->res_gm) (void)hipFree(c->res_gm);
    if (c->hold_word) (void)hipHostFree(c->hold_word);
    if (c->res_stamps) (void)hipFree(c->res_stamps);
    if (c->res_trace) (void)hipFree(c->res_trace);
    if (c->res_err) (void)hipHostFree(c->res_err);
    if (c->sr_dev) (void)hipFree(c->sr_dev);
    if (c->sr_mir) (void)hipHostFree(c->sr_mir);
    if (c->sr_hist) (void)hipFree(c->sr_hist);
    for (hipEvent_t e : c->sr_pend) (void)hipEventDestroy(e);
    for (hipEvent_t e : c->sr_evfree) (void)hipEventDestroy(e);
    double *bufs[] = {c->V, c->w, c->z, c->aux, c->dA, c->dB, c->x, c->b, c->vj, c->hlo, c->hhi, c->dh, c->zline,
                      c->red, c->hcol, c->ydev, c->hb, c->scal, c->Vb, c->gram_slab, c->gram_out};
    for (double *p : bufs)
        if (p) (void)hipFree(p);
    if (c->gram_pairs) (void)hipFree(c->gram_pairs);
    if (c->hcol_host) (void)hipHostFree(c->hcol_host);
    if (c->hall) (void)hipFree(c->hall);
    if (c->hallh) (void)hipHostFree(c->hallh);
    for (hipEvent_t e : c->ev_step)
        if (e) (void)hipEventDestroy(e);
    for (size_t k = 0; k < c->ev0.size(); ++k) {
        if (c->ev0[k]) (void)hipEventDestroy(c->ev0[k]);
        if (c->ev1[k]) (void)hipEventDestroy(c->ev1[k]);
    }
    if (c->st) (void)hipStreamDestroy(c->st);
    delete c;
    return GK_OK;
}

int gk_comm_unique_id(unsigned char id[128]) {
    ncclUniqueId u;
    NCCLCHK(ncclGetUniqueId(&u));
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
    std::memcpy(id, &u, 128);
    return GK_OK;
}

int gk_comm_init(gk_ctx *c, int nranks, int rank, int max_lines, const unsigned char id[128]) {
    if (c == nullptr || nranks < 1 || rank < 0 || rank >= nranks || max_lines < c->nlines)
        return set_err(GK_ERR_ARG, "bad comm args");
    graph_reset(c);
    HIPCHK(hipSetDevice(c->dev));
    c->nranks = nranks;
    c->rank = rank;
    c->max_lines = max_lines;
    c->min_lines = 0;
    set_geometry(c);
    // A 1-rank RCCL communicator is only built on request (GK_FORCE_RCCL=1): it
    // routes every collective through RCCL on one GPU (used by the tests).
    const char *force = std::getenv("GK_FORCE_RCCL");
    if (nranks > 1 || (force != nullptr && force[0] == '1')) {
        ncclUniqueId u;
        std::memcpy(&u, id, 128);
        ncclComm_t cm = nullptr;  // c->comm stays null when the init fails (gk_destroy, a later
        NCCLCHK(ncclCommInitRank(&cm, nranks, u, rank));  // gk_comm_init_xgmi)
        c->comm = cm;
        c->comm_ok = true;
    }
    return GK_OK;
}

int gk_group_create(int nranks, gk_group **out) {
    if (out == nullptr || nranks < 1 || nranks > LG_MAX) return set_err(GK_ERR_ARG, "bad group size");
    gk_group *g = new gk_group();
    g->n = nranks;
    g->members.assign(nranks, nullptr);
    g->ptrs.assign(nranks, nullptr);
    *out = g;
    return GK_OK;
}

int gk_group_destroy(gk_group *g) {
    delete g;
    return GK_OK;
}

int gk_comm_init_local(gk_ctx *c, gk_group *g, int rank, int max_lines) {
    if (c == nullptr || g == nullptr || rank < 0 || rank >= g->n || max_lines < c->nlines)
        return set_err(GK_ERR_ARG, "bad local comm args");
    graph_reset(c);
    HIPCHK(hipSetDevice(c->dev));
    c->nranks = g->n;
    c->rank = rank;
    c->max_lines = max_lines;
    c->min_lines = 0;
    set_geometry(c);
    c->lg = g;
    c->res_share = g->n;  // members may share one device: resident launches split its CUs
    HIPCHK(hipEventCreateWithFlags(&c->lev_a, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&c->lev_b, hipEventDisableTiming));
    if (hipMalloc(&c->lscratch, sizeof(double) * gk::NPMAX * 4) != hipSuccess)
        return set_err(GK_ERR_NOMEM, "local comm scratch");
    {
        std::lock_guard<std::mutex> lk(g->mu);
        g->members[rank] = c;
    }
    CHK(xs_alloc(c));
    c->comm_ok = true;
    return GK_OK;
}

int gk_comm_init_xgmi(gk_ctx *c, int nranks, int rank, int max_lines) {
    if (c == nullptr || nranks < 1 || nranks > gk::XS_MAXR || rank < 0 || rank >= nranks || max_lines < c->nlines)
        return set_err(GK_ERR_ARG, "bad xgmi comm args (nranks <= %d)", gk::XS_MAXR);
    graph_reset(c);
    HIPCHK(hipSetDevice(c->dev));
    if (c->comm != nullptr) {  // an RCCL communicator of an abandoned gk_comm_init: the exchange replaces it
        // abort, not destroy: ncclCommDestroy finalises collectively and can wait on
        // peers whose init failed or that have moved on; ncclCommAbort is local
        ncclCommAbort(c->comm);
        c->comm = nullptr;
        c->comm_ok = false;
    }
    c->nranks = nranks;
    c->rank = rank;
    c->max_lines = max_lines;
    c->min_lines = 0;
    set_geometry(c);
    return xs_alloc(c);  // comm_ok once gk_xchg_open has mapped the peers
}

int gk_xchg_handle(gk_ctx *c, unsigned char handle[64]) {
    if (c == nullptr || handle == nullptr) return set_err(GK_ERR_ARG, "null argument");
    CHK(xs_alloc(c));
    hipIpcMemHandle_t h;
    static_assert(sizeof(hipIpcMemHandle_t) == 64, "hipIpcMemHandle_t size");
    HIPCHK(hipIpcGetMemHandle(&h, c->xs_buf));
    std::memcpy(handle, &h, 64);
    return GK_OK;
}

int gk_xchg_open(gk_ctx *c, const unsigned char *handles) {
    if (c == nullptr || handles == nullptr) return set_err(GK_ERR_ARG, "null argument");
    if (c->nranks > gk::XS_MAXR) return set_err(GK_ERR_ARG, "device exchange supports <= %d ranks", gk::XS_MAXR);
    if (c->xs_ready) return set_err(GK_ERR_STATE, "exchange already open");
    CHK(xs_alloc(c));
    HIPCHK(hipSetDevice(c->dev));
    for (int r = 0; r < c->nranks; ++r) {
        if (r == c->rank) {
            c->xs_peers.p[r] = c->xs_buf;
            continue;
        }
        hipIpcMemHandle_t h;
        std::memcpy(&h, handles + 64 * (size_t)r, 64);
        void *p = nullptr;
        HIPCHK(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
        c->xs_mapped.push_back(p);
        c->xs_peers.p[r] = static_cast<gk::u64 *>(p);
    }
    graph_reset(c);  // captured steps hold the collective they were captured with
    c->xs_ready = true;
    c->xs_on = true;
    c->comm_ok = true;
    return GK_OK;
}

// Hardware queues HIP gives this process per device: GPU_MAX_HW_QUEUES, else
// HIP's default of 4.
int hw_queues() {
    const char *e = std::getenv("GPU_MAX_HW_QUEUES");
    const int q = (e != nullptr && *e != '\0') ? std::atoi(e) : 4;
    return q > 0 ? q : 4;
}

int gk_xchg_local(gk_ctx *c) {
    if (c == nullptr || c->lg == nullptr) return set_err(GK_ERR_STATE, "gk_xchg_local needs gk_comm_init_local");
    if (c->nranks > gk::XS_MAXR) return set_err(GK_ERR_ARG, "device exchange supports <= %d ranks", gk::XS_MAXR);
    std::lock_guard<std::mutex> lk(c->lg->mu);
    int same_dev = 0;
    for (int r = 0; r < c->nranks; ++r) {
        gk_ctx *o = c->lg->members[r];
        if (o == nullptr || o->xs_buf == nullptr)
            return set_err(GK_ERR_STATE, "rank %d of the group has not joined yet", r);
        same_dev += o->dev == c->dev;
    }
    // Every in-process rank on this device spins on its peers' granules from its
    // own stream: the streams must not share a hardware queue, or a spinning
    // exchange kernel can sit in front of its peer's kernel until the deadline
    // (seen with 4 ranks under HIP's default of 4 queues).  One more stream (the
    // null stream) may hold a queue too.
    const int q = hw_queues();
    if (same_dev + 1 > q)
        return set_err(GK_ERR_STATE,
                       "%d in-process ranks on device %d (+1 stream) need more than the %d hardware queues of this "
                       "process (GPU_MAX_HW_QUEUES): their spinning exchange kernels would deadlock; set "
                       "GPU_MAX_HW_QUEUES >= %d before the HIP runtime starts",
                       same_dev, c->dev, q, same_dev + 1);
    for (int r = 0; r < c->nranks; ++r) c->xs_peers.p[r] = c->lg->members[r]->xs_buf;
    graph_reset(c);
    c->xs_ready = true;
    c->xs_on = true;
    return GK_OK;
}

int gk_xchg_enable(gk_ctx *c, int on) {
    if (c == nullptr) return set_err(GK_ERR_ARG, "null context");
    graph_reset(c);
    if (on && !c->xs_ready) return set_err(GK_ERR_STATE, "exchange not open");
    if (on && c->xs_broken)
        return set_err(GK_ERR_STATE, "device exchange retired after a missed deadline (sequence numbers may "
                                     "differ between ranks)");
    if (!on && c->comm == nullptr && c->lg == nullptr && c->nranks > 1)
        return set_err(GK_ERR_STATE, "no RCCL or local communicator to fall back to");
    c->xs_on = on != 0;
    if (!c->xs_on && c->xs_err != nullptr) *c->xs_err = 0;  // a missed deadline does not outlive the switch
    return GK_OK;
}

namespace {
double host_hash(long long g, unsigned long long seed) {  // = gk::k_fill_hash
    unsigned long long z = (unsigned long long)g + seed * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z = z ^ (z >> 31);
    return (double)(z >> 11) * (2.0 / 9007199254740992.0) - 1.0;
}

int xs_selftest_body(gk_ctx *c, std::string &why) {
    const int R = c->nranks, me = c->rank;
    // element-wise sum of a short vector
    double hv[8];
    for (int k = 0; k < 8; ++k) hv[k] = (me + 1) * (k + 1) + 0.25 * k;
    double *d = slot(c, 3);
    HIPCHK(hipMemcpyAsync(d, hv, sizeof hv, hipMemcpyHostToDevice, c->st));
    CHK(allreduce(c, d, 8, true));
    // a partial slab: 5 partials of (rank+1) -> {5 * sum(rank+1), 0, 0, 0, 0}
    double hs[5];
    for (double &v : hs) v = me + 1.0;
    double *e = slot(c, 2);
    HIPCHK(hipMemcpyAsync(e, hs, sizeof hs, hipMemcpyHostToDevice, c->st));
    CHK(allreduce(c, e, 5));
    // broadcast from the last rank
    double hb[3] = {me + 0.5, -me - 0.5, 1e300 * (me + 1)};
    HIPCHK(hipMemcpyAsync(c->hb, hb, sizeof hb, hipMemcpyHostToDevice, c->st));
    CHK(bcast(c, c->hb, 3, R - 1));
    // halo lines of a globally indexed vector
    gk::k_fill_hash<<<c->nblk_stream, gk::TPB, 0, c->st>>>(c->vj, c->nloc, c->g0, 7);
    LAUNCHCHK();
    CHK(halo(c, c->vj));
    double rv[8], rs[5], rb[3];
    std::vector<double> lo(c->N), hi(c->N);
    HIPCHK(hipMemcpyAsync(rv, d, sizeof rv, hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipMemcpyAsync(rs, e, sizeof rs, hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipMemcpyAsync(rb, c->hb, sizeof rb, hipMemcpyDeviceToHost, c->st));
    if (me > 0) HIPCHK(hipMemcpyAsync(lo.data(), c->hlo, sizeof(double) * c->N, hipMemcpyDeviceToHost, c->st));
    if (me < R - 1) HIPCHK(hipMemcpyAsync(hi.data(), c->hhi, sizeof(double) * c->N, hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    if (*c->xs_err) {
        why = "missed the deadline waiting for " + xs_culprit(*c->xs_err);
        return GK_ERR_COMM;
    }
    for (int k = 0; k < 8; ++k) {
        double ex = 0.0;
        for (int r = 0; r < R; ++r) ex = ex + ((r + 1) * (k + 1) + 0.25 * k);
        if (rv[k] != ex) why = "vector all-reduce mismatch";
    }
    if (rs[0] != 5.0 * (R * (R + 1) / 2) || rs[1] != 0.0 || rs[4] != 0.0) why = "slab all-reduce mismatch";
    const int rt = R - 1;
    if (rb[0] != rt + 0.5 || rb[1] != -rt - 0.5 || rb[2] != 1e300 * (rt + 1)) why = "broadcast mismatch";
    for (int i = 0; i < c->N; ++i) {
        if (me > 0 && lo[i] != host_hash(c->g0 - c->N + i, 7)) why = "lower halo mismatch";
        if (me < R - 1 && hi[i] != host_hash(c->g0 + c->nloc + i, 7)) why = "upper halo mismatch";
    }
    return why.empty() ? GK_OK : GK_ERR_COMM;
}
}  // namespace

int gk_peer_info(int device, int peer, int *can_access, int *link_type, int *hops) {
    if (can_access == nullptr || link_type == nullptr || hops == nullptr) return set_err(GK_ERR_ARG, "null out");
    int n = 0;
    HIPCHK(hipGetDeviceCount(&n));
    if (device < 0 || peer < 0 || device >= n || peer >= n)
        return set_err(GK_ERR_ARG, "devices %d, %d outside 0..%d", device, peer, n - 1);
    *can_access = 1;
    *link_type = 0;
    *hops = 0;
    if (device == peer) return GK_OK;
    HIPCHK(hipDeviceCanAccessPeer(can_access, device, peer));
    unsigned lt = 0, hc = 0;
    HIPCHK(hipExtGetLinkTypeAndHopCount(device, peer, &lt, &hc));
    *link_type = (int)lt;
    *hops = (int)hc;
    return GK_OK;
}

int gk_xchg_selftest(gk_ctx *c, int timeout_ms) {
    CHK(check_ctx(c));
    if (!c->xs_ready) return set_err(GK_ERR_STATE, "exchange not open");
    HIPCHK(hipSetDevice(c->dev));
    {  // tests: this rank fails at once without taking part (its peers then miss their deadline)
        const char *f = std::getenv("GK_DEBUG_SELFTEST_FAIL");
        if (f != nullptr && f[0] != '\0' && std::atoi(f) == c->rank) {
            c->xs_on = false;
            graph_reset(c);
            if (c->comm == nullptr && c->lg == nullptr) c->comm_ok = c->nranks == 1;
            return set_err(GK_ERR_COMM, "device exchange self-test failed on rank %d: forced (GK_DEBUG_SELFTEST_FAIL)",
                           c->rank);
        }
    }
    const bool was_on = c->xs_on;
    const int t_keep = c->xs_timeout_ms;
    if (!was_on) graph_reset(c);  // graphs captured on another collective must not replay over this one
    c->xs_on = true;
    xs_set_timeout(c, timeout_ms > 0 ? timeout_ms : t_keep);
    std::string why;
    int rc = xs_selftest_body(c, why);
    if (rc == GK_ERR_HIP || rc == GK_ERR_ARG) why = g_err;
    xs_set_timeout(c, t_keep);
    if (rc != GK_OK) {
        (void)hipStreamSynchronize(c->st);
        *c->xs_err = 0;
        c->xs_on = false;
        graph_reset(c);  //  graphs captured over the exchange would replay its k_xchg nodes
        if (c->comm == nullptr && c->lg == nullptr) c->comm_ok = c->nranks == 1;
        return set_err(GK_ERR_COMM, "device exchange self-test failed on rank %d: %s", c->rank, why.c_str());
    }
    (void)was_on;
    return GK_OK;
}

int gk_comm_latency(gk_ctx *c, int iters, double *allreduce_us, double *halo_us) {
    CHK(check_ctx(c));
    if (iters < 1 || allreduce_us == nullptr || halo_us == nullptr) return set_err(GK_ERR_ARG, "bad arguments");
    *allreduce_us = *halo_us = 0.0;
    if (!collective(c)) return GK_OK;
    HIPCHK(hipSetDevice(c->dev));
    hipEvent_t e[3];
    for (auto &x : e) HIPCHK(hipEventCreate(&x));
    double *buf = slot(c, 0);
    const int count = std::max(1, c->np_pj);  // one projection's partial slab, as the launch path sends it
    int rc = allreduce(c, buf, count);         // warm: first-call setup stays out of the timing
    if (rc == GK_OK) rc = halo(c, c->w);
    if (rc == GK_OK) rc = hipEventRecord(e[0], c->st) == hipSuccess ? GK_OK : GK_ERR_HIP;
    for (int i = 0; i < iters && rc == GK_OK; ++i) rc = allreduce(c, buf, count);
    if (rc == GK_OK) rc = hipEventRecord(e[1], c->st) == hipSuccess ? GK_OK : GK_ERR_HIP;
    for (int i = 0; i < iters && rc == GK_OK; ++i) rc = halo(c, c->w);
    if (rc == GK_OK) rc = hipEventRecord(e[2], c->st) == hipSuccess ? GK_OK : GK_ERR_HIP;
    if (rc == GK_OK) rc = sync_st(c);
    float a = 0.f, b = 0.f;
    if (rc == GK_OK && (hipEventElapsedTime(&a, e[0], e[1]) != hipSuccess ||
                        hipEventElapsedTime(&b, e[1], e[2]) != hipSuccess))
        rc = set_err(GK_ERR_HIP, "event timing failed");
    for (auto &x : e) (void)hipEventDestroy(x);
    if (rc != GK_OK) return rc;
    *allreduce_us = 1e3 * a / iters;
    *halo_us = 1e3 * b / iters;
    return GK_OK;
}

int gk_comm_info(gk_ctx *c, int *kind, int *nranks_seen) {
    if (c == nullptr || kind == nullptr || nranks_seen == nullptr) return set_err(GK_ERR_ARG, "null argument");
    *kind = GK_COMM_NONE;
    *nranks_seen = 1;
    if (c->xs_on) {
        *kind = GK_COMM_XGMI;
        int k = 0;
        for (int r = 0; r < c->nranks; ++r) k += c->xs_peers.p[r] != nullptr;
        *nranks_seen = k;
    } else if (c->lg != nullptr) {
        *kind = GK_COMM_LOCAL;
        *nranks_seen = c->lg->n;
    } else if (c->comm != nullptr) {
        *kind = GK_COMM_RCCL;
        NCCLCHK(ncclCommCount(c->comm, nranks_seen));
    }
    return GK_OK;
}

int gk_local_size(gk_ctx *c, long long *nloc) {
    CHK(check_ctx(c));
    *nloc = c->nloc;
    return GK_OK;
}

// The short-recurrence solvers keep their vectors in the Krylov columns and their
// state on the device: any call that changes the operator data, the right-hand
// side or x, or that starts a GMRES cycle (which overwrites the columns), ends the
// running gk_sr_* solve -- later gk_sr_iterate / status / history refuse until the
// next gk_sr_start.
static void sr_invalidate(gk_ctx *c) { c->sr_solver = -1; }

int gk_set_precond(gk_ctx *c, int kind, const double *params, int nparams, int degree) {
    CHK(check_ctx(c));
    sr_invalidate(c);
    if (kind < GK_PREC_IDENTITY || kind > GK_PREC_CHEB) return set_err(GK_ERR_ARG, "bad precond kind %d", kind);
    if (kind != GK_PREC_IDENTITY && (params == nullptr || nparams < 2))
        return set_err(GK_ERR_ARG, "precond needs params(1:2)");
    if (kind == GK_PREC_CHEB && (degree < 1 || degree > 64)) return set_err(GK_ERR_ARG, "bad degree %d", degree);
    c->pkind = kind;
    if (params != nullptr && nparams >= 2) {
        c->p0 = params[0];
        c->p1 = params[1];
    }
    c->pdeg = degree;
    graph_reset(c);
    if (kind == GK_PREC_CHEB && std::fabs(c->p1 - c->p0) == 0.0)
        return set_err(GK_ERR_ARG, "Chebyshev interval is empty");
    return GK_OK;
}

int gk_set_rhs(gk_ctx *c, const double *b) {
    CHK(check_ctx(c));
    sr_invalidate(c);
    HIPCHK(hipSetDevice(c->dev));
    HIPCHK(hipMemcpyAsync(c->b, b, sizeof(double) * c->nloc, hipMemcpyHostToDevice, c->st));
    CHK(sync_st(c));
    c->beta0 = -1.0;
    return GK_OK;
}

int gk_set_rhs_ones(gk_ctx *c) {
    CHK(check_ctx(c));
    sr_invalidate(c);
    HIPCHK(hipSetDevice(c->dev));
    gk::k_fill<<<c->nblk_stream, gk::TPB, 0, c->st>>>(c->aux, 1.0, c->nloc);
    LAUNCHCHK();
    CHK(halo(c, c->aux));
    gk::StArgs a{};
    a.x = c->aux;
    a.y = c->b;
    CHK(stencil(c, gk::OP_PLAIN, gk::ACC_NONE, a));
    CHK(sync_st(c));
    c->beta0 = -1.0;
    return GK_OK;
}

int gk_rhs_norm(gk_ctx *c, double *beta0) {
    CHK(check_ctx(c));
    HIPCHK(hipSetDevice(c->dev));
    CHK(proj(c, gk::PJ_DOT, c->b, nullptr, c->b, nullptr, 0, slot(c, 0), nullptr, 1.0));
    CHK(allreduce(c, slot(c, 0), c->np_pj));
    CHK(finalize(c, slot(c, 0), c->np_pj, c->scal, 1));
    CHK(d2h_sync(c, beta0, c->scal, 1));
    c->beta0 = *beta0;
    return GK_OK;
}

int gk_zero_x(gk_ctx *c) {
    CHK(check_ctx(c));
    HIPCHK(hipSetDevice(c->dev));
    HIPCHK(hipMemsetAsync(c->x, 0, sizeof(double) * c->nloc, c->st));
    CHK(sync_st(c));
    return GK_OK;
}

int gk_get_x(gk_ctx *c, double *x) {
    CHK(check_ctx(c));
    HIPCHK(hipSetDevice(c->dev));
    HIPCHK(hipMemcpyAsync(x, c->x, sizeof(double) * c->nloc, hipMemcpyDeviceToHost, c->st));
    CHK(sync_st(c));
    return GK_OK;
}

int gk_get_basis(gk_ctx *c, int which, int col, double *out) {
    CHK(check_ctx(c));
    const double *base = which == 0 ? c->V : (which == 1 ? c->Vb : nullptr);
    const int ncol = which == 0 ? c->m + 1 : c->m;
    if (base == nullptr) return set_err(GK_ERR_ARG, "basis %d not available", which);
    if (col < 0 || col >= ncol) return set_err(GK_ERR_ARG, "bad column %d", col);
    HIPCHK(hipSetDevice(c->dev));
    HIPCHK(hipMemcpyAsync(out, base + (i64)col * c->ld, sizeof(double) * c->nloc, hipMemcpyDeviceToHost, c->st));
    CHK(sync_st(c));
    return GK_OK;
}

int gk_set_x(gk_ctx *c, const double *x) {
    CHK(check_ctx(c));
    sr_invalidate(c);
    HIPCHK(hipSetDevice(c->dev));
    HIPCHK(hipMemcpyAsync(c->x, x, sizeof(double) * c->nloc, hipMemcpyHostToDevice, c->st));
    CHK(sync_st(c));
    return GK_OK;
}

int gk_true_residual(gk_ctx *c, double *rel) {
    CHK(check_ctx(c));
    HIPCHK(hipSetDevice(c->dev));
    double b0;
    if (c->beta0 < 0) CHK(gk_rhs_norm(c, &b0));
    CHK(halo(c, c->x));
    gk::StArgs a{};
    a.x = c->x;
    a.in1 = c->b;
    a.y = c->aux;
    a.part = slot(c, 2);
    CHK(stencil(c, gk::OP_RESID, gk::ACC_NORM, a));
    CHK(allreduce(c, slot(c, 2), c->np_st));
    CHK(finalize(c, slot(c, 2), c->np_st, c->scal + 1, 1));
    double r;
    CHK(d2h_sync(c, &r, c->scal + 1, 1));
    *rel = r / c->beta0;
    return GK_OK;
}

// ------------------------------------------------------------------ MGS-R --

int gk_mgs_cycle_start(gk_ctx *c, double *beta) {
    CHK(check_ctx(c));
    sr_invalidate(c);
    HIPCHK(hipSetDevice(c->dev));
    if (c->pend_res_blk != 0 || c->pend_res_pf >= 0) {  // a step change requested mid-cycle (gk_set_tuning)
        if (c->pend_res_blk != 0) c->tune_res_blk = c->pend_res_blk;
        if (c->pend_res_pf >= 0) c->tune_res_pf = c->pend_res_pf;
        c->pend_res_blk = 0;
        c->pend_res_pf = -1;
        set_geometry(c);
        graph_reset(c);
    }
    CHK(op_precond(c, c->x, c->w, true, gk::ACC_NORM, nullptr, slot(c, 0)));
    CHK(allreduce(c, slot(c, 0), c->last_np));
    CHK(scale(c, c->V, c->w, slot(c, 0), c->last_np, c->hcol));
    CHK(d2h_sync(c, beta, c->hcol, 1));
    c->cycle_mgs = true;
    c->cycle_hh = false;
    return GK_OK;
}

int gk_mgs_step_async(gk_ctx *c, int j) {
    CHK(check_ctx(c));
    if (j < 1 || j > c->m) return set_err(GK_ERR_ARG, "step j=%d outside 1..%d", j, c->m);
    if (!c->cycle_mgs) return set_err(GK_ERR_STATE, "gk_mgs_step before gk_mgs_cycle_start");
    HIPCHK(hipSetDevice(c->dev));
    const i64 ld = c->ld;
    double *V = c->V;
    const int m2 = c->m + 2;
    double *hs = c->hall + (i64)(j - 1) * m2;  // H(1:j+1, j) of this step, on device
    c->prof_on_step = (j % c->prof_every) == 0;
    const int s0 = 0;
    ResPlan rp;
    const bool res = res_plan(c, rp);
    // w = M^-1 A V(:,j), fused with the first dot <w, V(:,1)>
    CHK(op_precond(c, V + (i64)(j - 1) * ld, c->w, false, gk::ACC_DOT, V, slot(c, s0)));
    int np = c->last_np;
    if (res) {  // the whole cascade + norm + scale as one resident launch
        // N ranks on the device exchange: the first dot's rank totals inside the launch
        // (GK_TUNE_RES_FOLD) instead of a k_xchg launch before it
        const bool fold = c->tune_res_fold && c->xs_on && c->nranks > 1;
        if (!fold) CHK(allreduce(c, slot(c, s0), np));
        CHK(res_step(c, j, rp, slot(c, s0), np, hs, c->hallh_dev + (i64)(j - 1) * m2, gk::RES_MGS, nullptr, -1,
                     fold ? RESF_PIN_LOCAL : 0));
        HIPCHK(hipEventRecord(c->ev_step[j], c->st));
        c->prof_on_step = true;
        return GK_OK;
    }
    // Launch path: RCCL ranks (or one rank with the resident step off) replay the
    // step's projection chain as a hipGraph captured at its first use (GK_TUNE_GRAPH).
    if (c->tune_graph && (c->lg == nullptr || c->xs_on)) {
        if (c->gkey != np) {
            graph_reset(c);
            c->gkey = np;
        }
        if ((int)c->gstep.size() < c->m + 1) c->gstep.resize(c->m + 1, nullptr);
        if (c->gstep[j] == nullptr) CHK(capture_step(c, j, np));
        if (c->gstep[j] != nullptr) {
            {
                ProfScope ps(c, GK_KID_GRAPH);
                if (c->xs_on && c->gxs[j] > 0) {  // the replay's exchanges continue this context's numbering
                    HIPCHK(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(c->xs_seqdev), (int)c->xs_seq, 1, c->st));
                    c->xs_seq += c->gxs[j];
                }
                HIPCHK(hipGraphLaunch(c->gstep[j], c->st));
            }
            HIPCHK(hipEventRecord(c->ev_step[j], c->st));
            c->prof_on_step = true;
            return GK_OK;
        }
    }
    CHK(mgs_chain(c, j, np));
    HIPCHK(hipEventRecord(c->ev_step[j], c->st));
    c->prof_on_step = true;
    return GK_OK;
}

// The host's per-step wait for the Hessenberg column.  Spinning on the event
// (default) keeps the wake-up off the critical path: a blocking wait sleeps
// in the driver and costs a scheduler wake-up per Arnoldi step, which a
// process that initialised another HIP user first (torch) was measured to
// pay -- 1024^2 cycles 37.0 -> 45.8 ms with identical kernel times.
int wait_step_event(gk_ctx *c, hipEvent_t e) {
    if (!c->tune_spin_wait) {
        HIPCHK(hipEventSynchronize(e));
        return GK_OK;
    }
    return spin_until(c, query_event, e, "Arnoldi step wait");
}

int gk_mgs_step_wait(gk_ctx *c, int j, double *hcol) {
    CHK(check_ctx(c));
    if (j < 1 || j > c->m) return set_err(GK_ERR_ARG, "step j=%d outside 1..%d", j, c->m);
    CHK(wait_step_event(c, c->ev_step[j]));
    CHK(res_check(c));
    CHK(xs_check(c));
    const volatile double *src = c->hallh + (i64)(j - 1) * (c->m + 2);
    for (int k = 0; k <= j; ++k) hcol[k] = src[k];
    return GK_OK;
}

int gk_mgs_step(gk_ctx *c, int j, double *hcol) {
    CHK(gk_mgs_step_async(c, j));
    return gk_mgs_step_wait(c, j, hcol);
}

int gk_update_x(gk_ctx *c, const double *y, int n_out) {
    CHK(check_ctx(c));
    if (n_out < 1 || n_out > c->m) return set_err(GK_ERR_ARG, "bad n_out %d", n_out);
    HIPCHK(hipSetDevice(c->dev));
    HIPCHK(hipMemcpyAsync(c->ydev, y, sizeof(double) * n_out, hipMemcpyHostToDevice, c->st));
    {
        ProfScope ps(c, GK_KID_UPDATE);
        gk::k_update_x<<<c->nblk_stream, gk::TPB, 0, c->st>>>(c->x, c->V, c->ld, c->ydev, n_out, c->nloc);
        LAUNCHCHK();
    }
    CHK(sync_st(c));
    if (c->prof) CHK(prof_harvest(c));
    return GK_OK;
}

int gk_mgs_verr(gk_ctx *c, int n_out, int zero_last, double *v_err) {
    CHK(check_ctx(c));
    if (n_out < 1 || n_out > c->m) return set_err(GK_ERR_ARG, "bad n_out %d", n_out);
    HIPCHK(hipSetDevice(c->dev));
    const int nc = n_out + 1;
    std::vector<double> G;
    CHK(gram(c, c->V, nc, G));
    if (zero_last)
        for (int i = 0; i < nc; ++i) {
            G[(size_t)(nc - 1) * nc + i] = 0.0;
            G[(size_t)i * nc + nc - 1] = 0.0;
        }
    // v_err(j+1) = sqrt(v_err(j)^2 + sum_{i<=j} 2 (V_i.V_{j+1})^2 + (V_{j+1}.V_{j+1}-1)^2)
    for (int k = 0; k <= c->m; ++k) v_err[k] = 0.0;
    for (int j = 1; j <= n_out; ++j) {
        double s = 0.0;
        for (int i = 1; i <= j; ++i) {
            const double d = G[(size_t)j * nc + (i - 1)];
            s = s + 2.0 * (d * d);
        }
        const double dd = G[(size_t)j * nc + j] - 1.0;
        s = s + dd * dd;
        v_err[j] = std::sqrt(v_err[j - 1] * v_err[j - 1] + s);
    }
    return GK_OK;
}

// ------------------------------------------------------------- Householder --

// GK_TUNE_HH_NORM_ORDER: the reflector norms in flang-rt's order -- a running sum over
// the whole vector, so one rank only (N ranks keep the tree).
static bool hh_seq_norms(const gk_ctx *c) { return c->tune_hh_norm_order != 0 && c->nranks == 1; }

static int hh_pivot(gk_ctx *c, int j, double *hostout, int nout) {
    // hb[0..j] = w(1:j+1) from the owning rank, broadcast
    const int root = owner_of(c, j);
    if (c->rank == root)
        HIPCHK(hipMemcpyAsync(c->hb, c->w + (0 - c->g0), sizeof(double) * (j + 1), hipMemcpyDeviceToDevice, c->st));
    CHK(bcast(c, c->hb, j + 1, root));
    return GK_OK;
    (void)hostout;
    (void)nout;
}

int gk_hh_cycle_start(gk_ctx *c, int precondition, double *g1) {
    CHK(check_ctx(c));
    sr_invalidate(c);
    HIPCHK(hipSetDevice(c->dev));
    if (c->nranks > 1 && c->rank == 0 && c->nloc < c->m + 2)
        return set_err(GK_ERR_ARG, "Householder path needs the first slab to hold m+2 unknowns");
    if (precondition) {
        CHK(op_precond(c, c->x, c->w, true, gk::ACC_NORM, nullptr, slot(c, 0)));
    } else {
        CHK(halo(c, c->x));
        gk::StArgs a{};
        a.x = c->x;
        a.in1 = c->b;
        a.y = c->w;
        a.part = slot(c, 0);
        CHK(stencil(c, gk::OP_RESID, gk::ACC_NORM, a));
    }
    CHK(allreduce(c, slot(c, 0), c->last_np));
    // GK_TUNE_HH_NORM_ORDER: beta = norm2(w) and norm2 of the fixed w in the reference's
    // order (gmres_hh.f90:250-253), one rank
    const bool seq = hh_seq_norms(c);
    if (seq) CHK(norm2_seq(c, c->w, c->nloc, slot(c, 0)));
    CHK(hh_pivot(c, 0, nullptr, 0));
    {
        ProfScope ps(c, GK_KID_OTHER);
        gk::k_hh_pivot<<<1, gk::TPB, 0, c->st>>>(c->hb, slot(c, 0), seq ? 1 : c->last_np, 0, c->hcol, c->scal + 2,
                                                 nullptr, seq ? 1 : 0);
        LAUNCHCHK();
        // w(1) = sign(beta,w(1)) + w(1); norm2(w)
        gk::k_hh_fix<<<c->nblk_stream, gk::TPB, 0, c->st>>>(c->w, c->nloc, c->g0, 0, 0, c->scal + 2, slot(c, 1));
        LAUNCHCHK();
    }
    if (seq) {
        CHK(norm2_seq(c, c->w, c->nloc, slot(c, 1)));
        CHK(scale(c, c->V, c->w, slot(c, 1), 1, nullptr, nullptr, nullptr, 0, true));
    } else {
        CHK(allreduce(c, slot(c, 1), c->nblk_stream));
        CHK(scale(c, c->V, c->w, slot(c, 1), c->nblk_stream, nullptr));
    }
    CHK(d2h_sync(c, g1, c->hcol, 1));
    c->cycle_hh = true;
    c->cycle_mgs = false;
    return GK_OK;
}

int gk_hh_step_async(gk_ctx *c, int j, int precondition) {
    CHK(check_ctx(c));
    if (j < 1 || j > c->m) return set_err(GK_ERR_ARG, "step j=%d outside 1..%d", j, c->m);
    if (!c->cycle_hh) return set_err(GK_ERR_STATE, "gk_hh_step before gk_hh_cycle_start");
    HIPCHK(hipSetDevice(c->dev));
    const i64 ld = c->ld;
    double *P = c->V;
    // The w-only resident variant folds the step's small launches into its chains
    // (GK_TUNE_HH_FUSE): the DOWN chain builds e_j itself (no k_set_unit), the UP
    // chain ends with the fix-up and P(:,j+1) = w/||w|| (no k_hh_fix, no k_scale).
    ResPlan rp;
    const bool res = res_plan(c, rp, true);
    const bool seq = hh_seq_norms(c);  // reference-order reflector norms: the unfused step
    const bool fuse = res && rp.wo && c->tune_hh_fuse != 0 && !seq;
    // v_j = e_j ; v_j = P_1 .. P_j e_j
    if (!fuse) {
        ProfScope ps(c, GK_KID_OTHER);
        gk::k_set_unit<<<c->nblk_stream, gk::TPB, 0, c->st>>>(c->vj, c->nloc, c->g0, j - 1, 1.0);
        LAUNCHCHK();
    }
    CHK(reflect_chain_down(c, c->vj, j, j - 1, fuse ? RESF_UNIT_INIT : 0));
    // w = M^-1 A v_j (or A v_j), fused with <w, P_1>
    int s0 = 0, s1 = 1;
    if (precondition) {
        CHK(op_precond(c, c->vj, c->w, false, gk::ACC_DOT, P, slot(c, s0)));
    } else {
        CHK(halo(c, c->vj));
        gk::StArgs a{};
        a.x = c->vj;
        a.y = c->w;
        a.vdot = P;
        a.part = slot(c, s0);
        CHK(stencil(c, gk::OP_PLAIN, gk::ACC_DOT, a));
    }
    int np = c->last_np;
    // N ranks on the device exchange: <w, P_1> summed across ranks inside the launch (GK_TUNE_RES_FOLD)
    const bool fold = res && c->tune_res_fold && c->xs_on && c->nranks > 1;
    if (fuse) {  // w = P_j .. P_1 w, ||w(j+1:n)||^2, the fix-up and P(:,j+1), one launch
        if (!fold) CHK(allreduce(c, slot(c, s0), np));
        CHK(res_step(c, j, rp, slot(c, s0), np, slot(c, s1), nullptr, gk::RES_HH_UP, c->w, -1,
                     RESF_CLOSE_HH | (fold ? RESF_PIN_LOCAL : 0)));
        // H(1:j+1, j) from hb (written by the owner rank's launch) on every rank
        CHK(bcast(c, c->hb, j + 1, owner_of(c, j)));
        {
            ProfScope ps(c, GK_KID_OTHER);
            const int m2 = c->m + 2;
            gk::k_hh_pivot<<<1, gk::TPB, 0, c->st>>>(c->hb, slot(c, s1), 1, j, c->hall + (i64)(j - 1) * m2,
                                                     c->scal + 2, c->hallh_dev + (i64)(j - 1) * m2);
            LAUNCHCHK();
        }
        HIPCHK(hipEventRecord(c->ev_step[j], c->st));
        return GK_OK;
    }
    if (res) {  // w = P_j .. P_1 w and ||w(j+1:n)||^2 as one resident launch
        if (!fold) CHK(allreduce(c, slot(c, s0), np));
        CHK(res_step(c, j, rp, slot(c, s0), np, slot(c, s1), nullptr, gk::RES_HH_UP, c->w, -1,
                     fold ? RESF_PIN_LOCAL : 0));
        std::swap(s0, s1);
        np = 1;  // slot s0[0]: the rank-summed total
    } else {
        // w = P_j .. P_1 w ; the last reflection also accumulates ||w(j+1:n)||^2
        for (int i = 1; i <= j; ++i) {
            CHK(allreduce(c, slot(c, s0), np));
            const double *va = P + (i64)(i - 1) * ld;
            if (i < j) {
                CHK(proj(c, gk::PJ_AXPY_DOT, c->w, va, P + (i64)i * ld, slot(c, s0), np, slot(c, s1), nullptr,
                         2.0));
            } else {
                CHK(proj(c, gk::PJ_AXPY_NORM, c->w, va, nullptr, slot(c, s0), np, slot(c, s1), nullptr, 2.0,
                         (i64)j - c->g0));
            }
            np = c->np_pj;
            std::swap(s0, s1);
        }
        CHK(allreduce(c, slot(c, s0), np));
    }
    if (seq) {  // tmp = norm2(w(j+1:n)) in the reference's order (gmres_hh.f90:307)
        CHK(norm2_seq(c, c->w + j, c->nloc - j, slot(c, s0)));
        np = 1;
    }
    CHK(hh_pivot(c, j, nullptr, 0));
    {
        ProfScope ps(c, GK_KID_OTHER);
        const int m2 = c->m + 2;
        gk::k_hh_pivot<<<1, gk::TPB, 0, c->st>>>(c->hb, slot(c, s0), np, j, c->hall + (i64)(j - 1) * m2,
                                                 c->scal + 2, c->hallh_dev + (i64)(j - 1) * m2, seq ? 1 : 0);
        LAUNCHCHK();
        gk::k_hh_fix<<<c->nblk_stream, gk::TPB, 0, c->st>>>(c->w, c->nloc, c->g0, j, j, c->scal + 2, slot(c, s1));
        LAUNCHCHK();
    }
    if (seq) {  // w = w / norm2(w) (gmres_hh.f90:315)
        CHK(norm2_seq(c, c->w, c->nloc, slot(c, s1)));
        CHK(scale(c, P + (i64)j * ld, c->w, slot(c, s1), 1, nullptr, nullptr, nullptr, 0, true));
    } else {
        CHK(allreduce(c, slot(c, s1), c->nblk_stream));
        CHK(scale(c, P + (i64)j * ld, c->w, slot(c, s1), c->nblk_stream, nullptr));
    }
    HIPCHK(hipEventRecord(c->ev_step[j], c->st));
    return GK_OK;
}

int gk_hh_step_wait(gk_ctx *c, int j, double *hcol) {
    return gk_mgs_step_wait(c, j, hcol);  // same per-step slot + event protocol
}

int gk_hh_step(gk_ctx *c, int j, int precondition, double *hcol) {
    CHK(gk_hh_step_async(c, j, precondition));
    return gk_hh_step_wait(c, j, hcol);
}

int gk_hh_update_x(gk_ctx *c, const double *y, int n_out) {
    CHK(check_ctx(c));
    if (n_out < 1 || n_out > c->m) return set_err(GK_ERR_ARG, "bad n_out %d", n_out);
    HIPCHK(hipSetDevice(c->dev));
    HIPCHK(hipMemcpyAsync(c->ydev, y, sizeof(double) * n_out, hipMemcpyHostToDevice, c->st));
    {
        ProfScope ps(c, GK_KID_OTHER);
        gk::k_set_prefix<<<c->nblk_stream, gk::TPB, 0, c->st>>>(c->w, c->nloc, c->g0, c->ydev, 0, n_out);
        LAUNCHCHK();
    }
    CHK(reflect_chain_down(c, c->w, n_out));
    {
        ProfScope ps(c, GK_KID_UPDATE);
        gk::k_add<<<c->nblk_stream, gk::TPB, 0, c->st>>>(c->x, c->w, c->nloc);
        LAUNCHCHK();
    }
    CHK(sync_st(c));
    if (c->prof) CHK(prof_harvest(c));
    return GK_OK;
}

int gk_hh_verr(gk_ctx *c, int n_out, double *v_err) {
    CHK(check_ctx(c));
    if (n_out < 1 || n_out > c->m) return set_err(GK_ERR_ARG, "bad n_out %d", n_out);
    HIPCHK(hipSetDevice(c->dev));
    if (c->Vb == nullptr) {
        if (hipMalloc(&c->Vb, sizeof(double) * (size_t)c->ld * c->m) != hipSuccess)
            return set_err(GK_ERR_NOMEM, "cannot allocate the verr basis");
    }
    for (int i = 1; i <= n_out; ++i) {
        double *col = c->Vb + (i64)(i - 1) * c->ld;
        gk::k_set_unit<<<c->nblk_stream, gk::TPB, 0, c->st>>>(col, c->nloc, c->g0, i - 1, 1.0);
        LAUNCHCHK();
        if (!verr_ref_order(c)) CHK(reflect_chain_down(c, col, i, i - 1));
    }
    if (verr_ref_order(c)) {  // :581-585 with the reference's dots, all chains level by level
        CHK(ensure_gram(c, n_out));
        ProfScope ps(c, GK_KID_OTHER);
        for (int s = 0; s < n_out; ++s) {
            gk::k_hh_rebuild_dot<<<(n_out - s + 63) / 64, 64, 0, c->st>>>(c->Vb, c->V, c->ld, c->nloc, s, n_out,
                                                                          c->gram_out);
            LAUNCHCHK();
            gk::k_hh_rebuild_upd<<<dim3(c->nblk_stream, n_out - s), gk::TPB, 0, c->st>>>(c->Vb, c->V, c->ld,
                                                                                       c->nloc, s, c->gram_out);
            LAUNCHCHK();
        }
    }
    std::vector<double> G;
    CHK(gram(c, c->Vb, n_out, G));
    for (int k = 0; k <= c->m; ++k) v_err[k] = 0.0;
    for (int i = 2; i <= n_out; ++i) {
        double s = 0.0;
        for (int jj = 1; jj < i; ++jj) {
            const double d = G[(size_t)(i - 1) * n_out + (jj - 1)];
            s = s + 2.0 * (d * d);
        }
        v_err[i - 1] = s;
    }
    return GK_OK;
}

int gk_apply(gk_ctx *c, int what, const double *in, double *out) {
    CHK(check_ctx(c));
    if (in == nullptr || out == nullptr || (what != 0 && what != 1)) return set_err(GK_ERR_ARG, "bad gk_apply args");
    HIPCHK(hipSetDevice(c->dev));
    c->cycle_mgs = c->cycle_hh = false;  // clobbers the work vectors
    if (what == 0) {
        HIPCHK(hipMemcpyAsync(c->vj, in, sizeof(double) * c->nloc, hipMemcpyHostToDevice, c->st));
        CHK(halo(c, c->vj));
        gk::StArgs a{};
        a.x = c->vj;
        a.y = c->w;
        CHK(stencil(c, gk::OP_PLAIN, gk::ACC_NONE, a));
    } else {
        HIPCHK(hipMemcpyAsync(c->z, in, sizeof(double) * c->nloc, hipMemcpyHostToDevice, c->st));
        if (c->pkind == GK_PREC_IDENTITY) {
            HIPCHK(hipMemcpyAsync(c->w, c->z, sizeof(double) * c->nloc, hipMemcpyDeviceToDevice, c->st));
        } else {
            CHK(precond_sweeps(c, c->w, gk::ACC_NONE, nullptr, nullptr));
        }
    }
    HIPCHK(hipMemcpyAsync(out, c->w, sizeof(double) * c->nloc, hipMemcpyDeviceToHost, c->st));
    CHK(sync_st(c));
    if (c->prof) CHK(prof_harvest(c));
    return GK_OK;
}

int gk_set_tuning(gk_ctx *c, int key, int value) {
    CHK(check_ctx(c));
    switch (key) {
        case GK_TUNE_PROJ_NT: c->tune_nt = value < 0 ? -1 : (value != 0); break;
        case GK_TUNE_PROJ_BLOCKS: c->tune_pj_blocks = value; break;
        case GK_TUNE_STENCIL_BLOCKS: c->tune_st_blocks = value; break;
        case GK_TUNE_CHEB_FUSED: c->tune_cheb_fused = value != 0; break;
        case GK_TUNE_PROJ_BLOCKED: c->tune_blocked = value != 0; break;
        case GK_TUNE_XCHG_TIMEOUT_MS:
            if (value < 1) return set_err(GK_ERR_ARG, "timeout must be >= 1 ms");
            xs_set_timeout(c, value);
            break;
        case GK_TUNE_RES: c->tune_res = value < 0 ? -1 : (value != 0); break;
        case GK_TUNE_RES_R2:
            if (value != 0 && value != 2 && value != 4 && value != 8 && value != 12)
                return set_err(GK_ERR_ARG, "resident cap must be 0 (auto), 2, 4, 8 or 12");
            c->tune_res_r2 = value;
            break;
        case GK_TUNE_RES_SHARE:
            if (value < 1) return set_err(GK_ERR_ARG, "share must be >= 1");
            c->res_share = value;
            break;
        case GK_TUNE_RES_LDS: c->tune_res_lds = value != 0; break;
        case GK_TUNE_RES_WONLY: c->tune_res_wonly = value < 0 ? -1 : (value != 0); break;
        case GK_TUNE_HH_FUSE: c->tune_hh_fuse = value != 0; break;
        case GK_TUNE_CHEB_STEN: c->tune_cheb_sten = value != 0; break;
        case GK_TUNE_SPIN_WAIT: c->tune_spin_wait = value != 0; break;
        case GK_TUNE_GRAPH: c->tune_graph = value != 0; break;
        case GK_TUNE_RES_QDEF: c->tune_res_qdef = value < 0 ? -1 : (value != 0); break;
        case GK_TUNE_RES_PC: c->tune_res_pc = value < 0 ? -1 : (value != 0); break;
        case GK_TUNE_RES_FOLD: c->tune_res_fold = value != 0; break;
        case GK_TUNE_WATCHDOG_MS: c->watchdog_ms = std::max(0, value); break;
        case GK_TUNE_HH_NORM_ORDER: c->tune_hh_norm_order = value != 0; break;
        // The blocked step reads Gram rows of earlier columns that only a blocked step of the
        // same cycle wrote: switching the step inside a cycle would use stale rows, so a change
        // requested while a cycle is open takes effect at the next gk_mgs_cycle_start.
        case GK_TUNE_RES_BLOCK:
            if (value != 1 && value != 2 && value != 4)
                return set_err(GK_ERR_ARG, "GK_TUNE_RES_BLOCK %d: blocks of 1 (strict MGS-R), 2 or 4 projections", value);
            if (c->cycle_mgs)
                c->pend_res_blk = value;
            else
                c->tune_res_blk = value;
            break;
        case GK_TUNE_SR_BLOCKS: c->tune_sr_blocks = std::max(0, value); break;
        case GK_TUNE_SR_TWO_LEVEL: c->tune_sr_two = value != 0; break;
        case GK_TUNE_RES_PF:
            if (c->cycle_mgs)
                c->pend_res_pf = value != 0;
            else
                c->tune_res_pf = value != 0;
            break;
        case GK_TUNE_VERR_ORDER: c->tune_verr_order = value != 0; break;
        case GK_TUNE_RES_TIMEOUT_MS:
            if (value < 1) return set_err(GK_ERR_ARG, "timeout must be >= 1 ms");
            c->res_timeout_ms = value;
            break;
        case GK_TUNE_PROJ_UNROLL:
            if (value != 0 && value != 2 && value != 4 && value != 8)
                return set_err(GK_ERR_ARG, "unroll must be 0 (auto), 2, 4 or 8");
            c->tune_unr = value;
            break;
        default: return set_err(GK_ERR_ARG, "unknown tuning key %d", key);
    }
    set_geometry(c);
    graph_reset(c);
    return GK_OK;
}

// ---------------------------------------------------------------- profiling --

int gk_profile_enable(gk_ctx *c, int enable) {
    CHK(check_ctx(c));
    if (!enable) CHK(prof_harvest(c));
    c->prof = enable != 0;
    c->prof_every = enable > 1 ? enable : 1;
    c->prof_on_step = true;
    return GK_OK;
}

int gk_profile_reset(gk_ctx *c) {
    CHK(check_ctx(c));
    CHK(prof_harvest(c));
    for (int k = 0; k < GK_NKID; ++k) {
        c->prof_ms[k] = 0.0;
        c->prof_n[k] = 0;
    }
    return GK_OK;
}

int gk_profile_read(gk_ctx *c, int kid, double *total_ms, long long *launches) {
    CHK(check_ctx(c));
    if (kid < 0 || kid >= GK_NKID) return set_err(GK_ERR_ARG, "bad kernel id");
    CHK(prof_harvest(c));
    *total_ms = c->prof_ms[kid];
    *launches = c->prof_n[kid];
    return GK_OK;
}

int gk_profile_res_wg(gk_ctx *c, int which, double *pass_ms, double *wait_ms, int maxwg, int *nwg) {
    CHK(check_ctx(c));
    if (which < 0 || which > 2 || pass_ms == nullptr || wait_ms == nullptr || nwg == nullptr || maxwg < 1)
        return set_err(GK_ERR_ARG, "bad arguments");
    *nwg = 0;
    if (c->res_stamps == nullptr) return GK_OK;
    HIPCHK(hipSetDevice(c->dev));
    std::vector<gk::u64> h(4 * (size_t)gk::RGMAX);
    HIPCHK(hipMemcpyAsync(h.data(), c->res_stamps + (size_t)which * 4 * gk::RGMAX, sizeof(gk::u64) * h.size(),
                          hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    const double tpm = (double)c->xs_tick_per_ms;
    int g = 0;
    for (int b = 0; b < gk::RGMAX && g < maxwg; ++b)
        if (h[4 * b + 3] > 0) {  // workgroups that ran, in blockIdx order
            pass_ms[g] = (double)h[4 * b] / tpm;
            wait_ms[g] = (double)h[4 * b + 1] / tpm;
            ++g;
        }
    *nwg = g;
    return GK_OK;
}

int gk_profile_res_trace(gk_ctx *c, int arm, int j, int mode, unsigned long long *out, int maxwg, int maxx,
                         int *nwg, int *nx, double *tick_per_ms) {
    CHK(check_ctx(c));
    HIPCHK(hipSetDevice(c->dev));
    const size_t words = (size_t)gk::RGMAX * gk::RES_TRACE_X * 2;
    if (arm == 1) {
        if (mode != gk::RES_MGS || j < 1) return set_err(GK_ERR_ARG, "trace: MGS-R step launches (mode 0), j >= 1");
        if (c->res_trace == nullptr) HIPCHK(hipMalloc(&c->res_trace, sizeof(gk::u64) * words));
        HIPCHK(hipMemsetAsync(c->res_trace, 0, sizeof(gk::u64) * words, c->st));
        HIPCHK(hipStreamSynchronize(c->st));
        c->res_trace_j = j;
        c->res_trace_mode = mode;
        c->res_trace_g = c->res_trace_np = 0;
        return GK_OK;
    }
    if (arm == 0) {
        c->res_trace_mode = -1;
        return GK_OK;
    }
    if (out == nullptr || nwg == nullptr || nx == nullptr || tick_per_ms == nullptr || maxwg < 1 || maxx < 1)
        return set_err(GK_ERR_ARG, "bad arguments");
    *nwg = *nx = 0;
    *tick_per_ms = (double)c->xs_tick_per_ms;
    if (c->res_trace == nullptr || c->res_trace_g == 0) return GK_OK;
    std::vector<gk::u64> h(words);
    HIPCHK(hipMemcpyAsync(h.data(), c->res_trace, sizeof(gk::u64) * words, hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    const int G = std::min(c->res_trace_g, maxwg), X = std::min({c->res_trace_np, maxx, gk::RES_TRACE_X});
    for (int b = 0; b < G; ++b)
        for (int x = 0; x < X; ++x)
            for (int k = 0; k < 2; ++k)
                out[((size_t)b * X + x) * 2 + k] = h[((size_t)b * gk::RES_TRACE_X + x) * 2 + k];
    *nwg = G;
    *nx = X;
    return GK_OK;
}

int gk_profile_res_split(gk_ctx *c, int mode, int which, double *pass_ms, double *wait_ms, double *total_ms,
                         long long *launches) {
    CHK(check_ctx(c));
    if (which < 0 || which > 2) return set_err(GK_ERR_ARG, "which must be 0 (MGS), 1 (HH up) or 2 (HH down)");
    HIPCHK(hipSetDevice(c->dev));
    const size_t bytes = sizeof(gk::u64) * 4 * 3 * gk::RGMAX;
    if (mode == 1 || mode == 2) {  // enable (and zero) / reset
        if (c->res_stamps == nullptr) HIPCHK(hipMalloc(&c->res_stamps, bytes));
        HIPCHK(hipMemsetAsync(c->res_stamps, 0, bytes, c->st));
        HIPCHK(hipStreamSynchronize(c->st));
        c->res_split = true;
    } else if (mode == 0) {
        c->res_split = false;
    }
    if (pass_ms == nullptr || wait_ms == nullptr || total_ms == nullptr || launches == nullptr) return GK_OK;
    *pass_ms = *wait_ms = *total_ms = 0.0;
    *launches = 0;
    if (c->res_stamps == nullptr) return GK_OK;
    std::vector<gk::u64> h(4 * (size_t)gk::RGMAX);
    HIPCHK(hipMemcpyAsync(h.data(), c->res_stamps + (size_t)which * 4 * gk::RGMAX, sizeof(gk::u64) * h.size(),
                          hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    // mean over the workgroups that ran (slot launches > 0), in ms of wall clock
    double sp = 0, sw = 0, st = 0;
    int g = 0;
    long long nl = 0;
    for (int b = 0; b < gk::RGMAX; ++b)
        if (h[4 * b + 3] > 0) {
            sp += (double)h[4 * b];
            sw += (double)h[4 * b + 1];
            st += (double)h[4 * b + 2];
            nl = std::max<long long>(nl, (long long)h[4 * b + 3]);
            ++g;
        }
    if (g > 0) {
        const double tpm = (double)c->xs_tick_per_ms;
        *pass_ms = sp / g / tpm;
        *wait_ms = sw / g / tpm;
        *total_ms = st / g / tpm;
    }
    *launches = nl;
    return GK_OK;
}

int gk_debug_hold_stream(gk_ctx *c, int hold) {
    if (c == nullptr) return set_err(GK_ERR_ARG, "null context");
    HIPCHK(hipSetDevice(c->dev));
    if (c->hold_word == nullptr) {
        HIPCHK(hipHostMalloc((void **)&c->hold_word, sizeof(unsigned), hipHostMallocMapped));
        HIPCHK(hipHostGetDevicePointer((void **)&c->hold_word_dev, c->hold_word, 0));
        *c->hold_word = 0;
    }
    if (hold) {
        if (c->broken) return set_err(GK_ERR_STATE, "context broken");
        __atomic_store_n(c->hold_word, 0u, __ATOMIC_RELEASE);
        HIPCHK(hipStreamWaitValue32(c->st, c->hold_word_dev, 1u, hipStreamWaitValueGte, 0xFFFFFFFFu));
    } else {
        __atomic_store_n(c->hold_word, 1u, __ATOMIC_RELEASE);
    }
    return GK_OK;
}

int gk_sync(gk_ctx *c) {
    CHK(check_ctx(c));
    HIPCHK(hipSetDevice(c->dev));
    CHK(sync_st(c));
    if (c->prof) CHK(prof_harvest(c));
    return GK_OK;
}

int gk_res_plan_query(long long nloc, int cus, int share, int hh, int nt, int block, long long *info) {
    if (info == nullptr || nloc < 2 || cus < 1 || share < 1 || (block != 1 && block != 2 && block != 4))
        return set_err(GK_ERR_ARG, "bad plan query");
    const int gmax = std::max(1, std::min(gk::RGMAX, cus / share));
    ResPlan p;
    plan_resident(nloc, gmax, RES_R2_BIG, 1, -1, hh != 0, nt < 0 ? nt_auto_for(nloc) : nt != 0, p, -1, block);
    plan_info(p, true, info);
    return GK_OK;
}

int gk_res_info(gk_ctx *c, int hh, long long *info) {
    CHK(check_ctx(c));
    if (info == nullptr) return set_err(GK_ERR_ARG, "null info");
    ResPlan p;
    const bool on = res_plan(c, p, hh != 0);
    plan_info(p, on, info);
    // op_precond_sten's conditions, without its collective (the smallest slab of
    // a multi-rank context is gathered at its first solve)
    int cs = c->pkind == GK_PREC_CHEB && c->tune_cheb_sten && c->pdeg <= gk::CF_LMAX && c->N >= gk::CF_PTS &&
             c->tune_cheb_fused && c->N % 2 == 0 &&
             (i64)c->N * std::max(c->nlines, c->max_lines) * 8 < (1LL << 31);
    if (cs && collective(c) && c->nranks > 1) cs = c->min_lines == 0 ? -1 : (c->min_lines >= c->pdeg + 1 ? 1 : 0);
    info[RPI_CHEB_STEN] = cs;
    return GK_OK;
}

}  // extern "C"

// ------------------------------------------------- stateless kernel API ----

namespace {
// Device scratch for the stateless calls: NSLOT partial slabs + a scalar area.
double *g_scratch[64] = {nullptr};

int stateless_ctx(gk_ctx &c, int N, int nlines, i64 n, void *stream) {
    int dev = 0;
    HIPCHK(hipGetDevice(&dev));
    if (dev < 0 || dev >= 64) return set_err(GK_ERR_ARG, "device id %d", dev);
    if (g_scratch[dev] == nullptr) {
        if (hipMalloc(&g_scratch[dev], sizeof(double) * (NSLOT * gk::NPMAX + 64)) != hipSuccess)
            return set_err(GK_ERR_NOMEM, "scratch allocation failed");
    }
    c.dev = dev;
    c.N = N;
    c.nlines = nlines;
    c.nloc = n;
    c.max_lines = nlines;
    c.st = reinterpret_cast<hipStream_t>(stream);
    c.red = g_scratch[dev];
    c.scal = g_scratch[dev] + NSLOT * gk::NPMAX;
    set_geometry(&c);
    return GK_OK;
}

void release_stateless(gk_ctx &c) {
    // nothing owned: keep the destructor-free fields from being freed
    c.red = nullptr;
    c.scal = nullptr;
    c.st = nullptr;
}

bool aligned16(const void *p) { return p == nullptr || (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }
}  // namespace

extern "C" {

int gk_poisson5(int nside, int nlines, const double *x, const double *hlo, const double *hhi, double *y,
                void *stream) {
    if (nside < 2 || nlines < 1 || x == nullptr || y == nullptr) return set_err(GK_ERR_ARG, "bad poisson5 args");
    if (!aligned16(x) || !aligned16(y) || !aligned16(hlo) || !aligned16(hhi))
        return set_err(GK_ERR_ARG, "device pointers must be 16-byte aligned");
    gk_ctx c;
    CHK(stateless_ctx(c, nside, nlines, (i64)nside * nlines, stream));
    gk::StArgs a{};
    a.x = x;
    a.y = y;
    a.N = nside;
    a.nlines = nlines;
    a.JT = c.JT;
    a.hlo = hlo;
    a.hhi = hhi;
    int rc = (c.vec == 2) ? launch_stencil_v<2, gk::OP_PLAIN, gk::ACC_NONE>(&c, a)
                          : launch_stencil_v<1, gk::OP_PLAIN, gk::ACC_NONE>(&c, a);
    release_stateless(c);
    return rc;
}

int gk_precond_apply(int nside, int kind, const double *params, int degree, const double *r, double *z,
                     double *scratch, void *stream) {
    if (nside < 2 || r == nullptr || z == nullptr) return set_err(GK_ERR_ARG, "bad precond args");
    if (!aligned16(r) || !aligned16(z) || !aligned16(scratch))
        return set_err(GK_ERR_ARG, "device pointers must be 16-byte aligned");
    const i64 n = (i64)nside * nside;
    gk_ctx c;
    CHK(stateless_ctx(c, nside, nside, n, stream));
    int rc = gk_set_precond(&c, kind, params, params ? 2 : 0, degree);
    if (rc == GK_OK && kind == GK_PREC_IDENTITY) {
        rc = hipMemcpyAsync(z, r, sizeof(double) * n, hipMemcpyDeviceToDevice, c.st) == hipSuccess
                 ? GK_OK
                 : set_err(GK_ERR_HIP, "copy failed");
    } else if (rc == GK_OK) {
        if (scratch == nullptr && kind == GK_PREC_CHEB) {
            rc = set_err(GK_ERR_ARG, "Chebyshev needs 3 scratch vectors");
        } else {
            // op_precond expects z = A v already formed for a step; here the input
            // IS the residual, so run the preconditioner sweeps directly on r.
            c.z = const_cast<double *>(r);
            c.aux = scratch;
            c.dA = scratch ? scratch + n : nullptr;
            c.dB = scratch ? scratch + 2 * n : nullptr;
            rc = precond_sweeps(&c, z, gk::ACC_NONE, nullptr, nullptr);
        }
    }
    c.z = c.aux = c.dA = c.dB = nullptr;
    release_stateless(c);
    return rc;
}

int gk_mgs_project(long long n, double *w, const double *va, double *result, void *stream) {
    if (n < 1 || w == nullptr || va == nullptr || result == nullptr) return set_err(GK_ERR_ARG, "bad args");
    if (!aligned16(w) || !aligned16(va)) return set_err(GK_ERR_ARG, "device pointers must be 16-byte aligned");
    gk_ctx c;
    CHK(stateless_ctx(c, 2, 1, n, stream));
    int rc = GK_OK;
    if (hipMemsetAsync(result, 0, sizeof(double), c.st) != hipSuccess) rc = set_err(GK_ERR_HIP, "memset");
    if (rc == GK_OK) rc = proj(&c, gk::PJ_DOT, w, nullptr, va, nullptr, 0, slot(&c, 0), nullptr, 1.0);
    if (rc == GK_OK) rc = proj(&c, gk::PJ_AXPY, w, va, nullptr, slot(&c, 0), c.np_pj, nullptr, result, 1.0);
    release_stateless(c);
    return rc;
}

int gk_dot(long long n, const double *a, const double *b, double *result, void *stream) {
    if (n < 1 || a == nullptr || b == nullptr || result == nullptr) return set_err(GK_ERR_ARG, "bad args");
    if (!aligned16(a) || !aligned16(b)) return set_err(GK_ERR_ARG, "device pointers must be 16-byte aligned");
    gk_ctx c;
    CHK(stateless_ctx(c, 2, 1, n, stream));
    int rc = proj(&c, gk::PJ_DOT, const_cast<double *>(a), nullptr, b, nullptr, 0, slot(&c, 0), nullptr, 1.0);
    if (rc == GK_OK) rc = finalize(&c, slot(&c, 0), c.np_pj, result, 0);
    release_stateless(c);
    return rc;
}

}  // extern "C"

// ------------------------------------------------------------------ Lanczos --

namespace {
// Number of eigenvalues of the symmetric tridiagonal (a, b) smaller than x (Sturm count).
int sturm_count(const std::vector<double> &a, const std::vector<double> &b, double x) {
    int cnt = 0;
    double q = 1.0;
    for (size_t i = 0; i < a.size(); ++i) {
        const double bb = i ? b[i - 1] * b[i - 1] : 0.0;
        q = a[i] - x - (i ? bb / q : 0.0);
        if (q == 0.0) q = -1e-300;
        if (q < 0.0) ++cnt;
    }
    return cnt;
}

double tridiag_eig(const std::vector<double> &a, const std::vector<double> &b, int which) {
    double lo = a[0], hi = a[0];
    for (size_t i = 0; i < a.size(); ++i) {
        const double r = (i ? std::fabs(b[i - 1]) : 0.0) + (i + 1 < a.size() ? std::fabs(b[i]) : 0.0);
        lo = std::min(lo, a[i] - r);
        hi = std::max(hi, a[i] + r);
    }
    for (int it = 0; it < 200; ++it) {  // bisection on the Sturm count
        const double mid = 0.5 * (lo + hi);
        if (sturm_count(a, b, mid) > which) hi = mid; else lo = mid;
    }
    return 0.5 * (lo + hi);
}

int dot_host(gk_ctx *c, const double *a, const double *b, double *out) {
    CHK(proj(c, gk::PJ_DOT, const_cast<double *>(a), nullptr, b, nullptr, 0, slot(c, 3), nullptr, 1.0));
    CHK(allreduce(c, slot(c, 3), c->np_pj));
    CHK(finalize(c, slot(c, 3), c->np_pj, c->scal + 6, 0));
    return d2h_sync(c, out, c->scal + 6, 1);
}

int axpy_host(gk_ctx *c, double *y, double a, const double *x) {
    gk::k_axpy_host<<<c->nblk_stream, gk::TPB, 0, c->st>>>(y, a, x, c->nloc);
    LAUNCHCHK();
    return GK_OK;
}
}  // namespace

extern "C" int gk_lanczos_bounds(gk_ctx *c, int k, double *lmin, double *lmax) {
    CHK(check_ctx(c));
    if (k < 2 || k > 1000 || lmin == nullptr || lmax == nullptr) return set_err(GK_ERR_ARG, "bad Lanczos args");
    HIPCHK(hipSetDevice(c->dev));
    c->cycle_mgs = c->cycle_hh = false;  // uses the work vectors
    double *qprev = c->dA, *q = c->dB, *w = c->vj;
    gk::k_fill_hash<<<c->nblk_stream, gk::TPB, 0, c->st>>>(q, c->nloc, c->g0, 12345ull);
    LAUNCHCHK();
    HIPCHK(hipMemsetAsync(qprev, 0, sizeof(double) * c->nloc, c->st));
    double nq;
    CHK(dot_host(c, q, q, &nq));
    CHK(axpy_host(c, q, 1.0 / std::sqrt(nq) - 1.0, q));  // q /= ||q||
    std::vector<double> al, be;
    double beta = 0.0;
    for (int it = 0; it < k; ++it) {
        CHK(halo(c, q));
        gk::StArgs a{};
        a.x = q;
        a.y = w;
        CHK(stencil(c, gk::OP_PLAIN, gk::ACC_NONE, a));   // w = A q
        if (beta != 0.0) CHK(axpy_host(c, w, -beta, qprev));
        double alpha;
        CHK(dot_host(c, w, q, &alpha));
        CHK(axpy_host(c, w, -alpha, q));
        double b2;
        CHK(dot_host(c, w, w, &b2));
        al.push_back(alpha);
        beta = std::sqrt(b2);
        if (beta == 0.0 || it == k - 1) break;
        be.push_back(beta);
        std::swap(qprev, q);                                // q_{j-1} <- q_j
        HIPCHK(hipMemcpyAsync(q, w, sizeof(double) * c->nloc, hipMemcpyDeviceToDevice, c->st));
        CHK(axpy_host(c, q, 1.0 / beta - 1.0, q));          // q_{j+1} = w / beta
    }
    be.resize(al.size() > 0 ? al.size() - 1 : 0);
    *lmin = tridiag_eig(al, be, 0);
    *lmax = tridiag_eig(al, be, (int)al.size() - 1);
    CHK(sync_st(c));
    return GK_OK;
}

// ------------------------------------------- device vector primitives -------
// Short-recurrence solvers (pcg_omp src/cg.f90:154-234, pbicgstab_omp
// src/bicgstab.f90:91-182) on context-resident vectors: id 0 = x, 1 = b,
// 2 .. m+2 = scratch (the Krylov columns).

namespace {
double *vec_of(gk_ctx *c, int id) {
    if (id == GK_VEC_X) return c->x;
    if (id == GK_VEC_B) return c->b;
    if (id >= 2 && id <= c->m + 2) return c->V + (i64)(id - 2) * c->ld;
    return nullptr;
}
}  // namespace

extern "C" {

int gk_vec_count(gk_ctx *c, int *count) {
    CHK(check_ctx(c));
    *count = c->m + 3;
    return GK_OK;
}

int gk_vec_apply(gk_ctx *c, int what, int in, int out) {
    CHK(check_ctx(c));
    double *vi = vec_of(c, in), *vo = vec_of(c, out);
    if (vi == nullptr || vo == nullptr || in == out || (what != 0 && what != 1))
        return set_err(GK_ERR_ARG, "bad gk_vec_apply(%d, %d, %d)", what, in, out);
    HIPCHK(hipSetDevice(c->dev));
    c->cycle_mgs = c->cycle_hh = false;
    if (what == 0) {
        CHK(halo(c, vi));
        gk::StArgs a{};
        a.x = vi;
        a.y = vo;
        return stencil(c, gk::OP_PLAIN, gk::ACC_NONE, a);
    }
    if (c->pkind == GK_PREC_IDENTITY) {
        HIPCHK(hipMemcpyAsync(vo, vi, sizeof(double) * c->nloc, hipMemcpyDeviceToDevice, c->st));
        return GK_OK;
    }
    HIPCHK(hipMemcpyAsync(c->z, vi, sizeof(double) * c->nloc, hipMemcpyDeviceToDevice, c->st));
    return precond_sweeps(c, vo, gk::ACC_NONE, nullptr, nullptr);
}

int gk_vec_dot(gk_ctx *c, int a, int b, double *result) {
    CHK(check_ctx(c));
    double *va = vec_of(c, a), *vb = vec_of(c, b);
    if (va == nullptr || vb == nullptr || result == nullptr) return set_err(GK_ERR_ARG, "bad gk_vec_dot");
    HIPCHK(hipSetDevice(c->dev));
    return dot_host(c, va, vb, result);
}

int gk_vec_lincomb(gk_ctx *c, int form, int out, int a, int b, int cc, double s1, double s2) {
    CHK(check_ctx(c));
    double *vo = vec_of(c, out);
    const double *va = vec_of(c, a), *vb = vec_of(c, b), *vc = vec_of(c, cc);
    const bool need_a = form != GK_LC_ZERO, need_b = form == GK_LC_AXPY || form == GK_LC_AXPY2 ||
                                                    form == GK_LC_XPAYMZ;
    const bool need_c = form == GK_LC_AXPY2 || form == GK_LC_XPAYMZ;
    if (vo == nullptr || form < 0 || form > GK_LC_ZERO || (need_a && va == nullptr) || (need_b && vb == nullptr) ||
        (need_c && vc == nullptr))
        return set_err(GK_ERR_ARG, "bad gk_vec_lincomb");
    HIPCHK(hipSetDevice(c->dev));
    gk::k_lincomb<<<c->nblk_stream, gk::TPB, 0, c->st>>>(form, vo, va, vb, vc, s1, s2, c->nloc);
    LAUNCHCHK();
    return GK_OK;
}

}  // extern "C"

// ------------------------------------- fused short-recurrence solvers -------
// pcg_omp (src/cg.f90:154-234) and pbicgstab_omp (src/bicgstab.f90:91-182) with
// every scalar on the device (gk_sr.hpp).  Vectors: Krylov columns 0..7 and the
// work vectors w, vj (free between GMRES cycles).  p and ap alternate between two
// buffers by iteration parity: the line march reads them with their neighbour
// lines while it writes the next ones.

namespace {
constexpr int SR_GRAPH_ITERS = 16;  // iterations per captured graph (even: the parity returns to 0)

struct SrVecs {
    double *r, *z, *r0, *p[2], *ap[2], *s, *as, *z1, *z2;
    double *rr[2];  // two-level PCG: r by iteration parity (the pass reads r around its lines while it writes the next)
};

SrVecs sr_vecs(gk_ctx *c) {
    auto col = [&](int k) { return c->V + (i64)k * c->ld; };
    SrVecs v{};
    v.r = col(0);
    v.z = col(1);   // PCG
    v.r0 = col(1);  // BiCGSTAB
    v.p[0] = col(2);
    v.p[1] = col(3);
    v.ap[0] = col(4);
    v.ap[1] = col(5);
    v.s = col(6);
    v.as = col(7);
    v.z1 = c->w;
    v.z2 = c->vj;
    v.rr[0] = col(0);
    v.rr[1] = col(6);  // s: unused by PCG
    return v;
}

bool sr_slabs(const gk_ctx *c) { return collective(c) && c->nranks > 1; }

gk::SrArgs sr_args(gk_ctx *c) {
    gk::SrArgs a{};
    a.sd = c->sr_dev;
    a.hist = c->sr_hist;
    a.mir = c->sr_mir_dev;
    a.part0 = slot(c, 0);
    a.part1 = slot(c, 1);
    a.zl = c->zline;
    a.N = c->N;
    a.nlines = c->nlines;
    a.JT = c->sr_JT;
    // cbpr2 coefficients exactly as chebyshev.f90:19-25 (precond_sweeps)
    const double cc = (c->p1 - c->p0) / 2.0, d = (c->p1 + c->p0) / 2.0;
    double al = 1.0 / d;
    double be = cc * al / 2.0;
    be = be * be;
    al = 1.0 / (d - be);
    a.cd = d;
    a.ca = al;
    return a;
}

// N ranks: the partial slab(s) are all-reduced, then k_sr_fin runs the finaliser.
int sr_fin_after(gk_ctx *c, int fin, int np, bool two) {
    if (fin == gk::FIN_NONE) return GK_OK;
    if (sr_slabs(c)) {
        CHK(allreduce(c, slot(c, 0), np));
        if (two) CHK(allreduce(c, slot(c, 1), np));
    }
    gk::k_sr_fin<<<1, gk::TPB, 0, c->st>>>(fin, c->sr_dev, slot(c, 0), slot(c, 1), np, c->sr_hist, c->sr_mir_dev);
    LAUNCHCHK();
    return GK_OK;
}

template <int K>
int sr_march(gk_ctx *c, gk::SrArgs a, int fin) {
    constexpr int NIN = gk::sr_nin<K>();
    const bool slabs = sr_slabs(c);
    if (slabs) {  // one halo line of every operand input (the operand is formed on load)
        const bool has_lo = c->rank > 0, has_hi = c->rank < c->nranks - 1;
        const double *in[3] = {a.in0, a.in1, a.in2};
        for (int v = 0; v < NIN; ++v) {
            double *lo = c->dh + (i64)(2 * v) * gk::CF_HMAX * c->N;
            double *hi = c->dh + (i64)(2 * v + 1) * gk::CF_HMAX * c->N;
            CHK(halo_lines(c, in[v], 1, lo, hi));
            a.lo[v] = has_lo ? lo : nullptr;
            a.hi[v] = has_hi ? hi : nullptr;
        }
    }
    a.fin = slabs ? gk::FIN_NONE : fin;
    {
        ProfScope ps(c, GK_KID_SR + K);
        if (c->vec == 2)
            gk::k_sr_march<2, K><<<c->sr_sgrid, gk::TPB, 0, c->st>>>(a);
        else
            gk::k_sr_march<1, K><<<c->sr_sgrid, gk::TPB, 0, c->st>>>(a);
        LAUNCHCHK();
    }
    if (slabs) CHK(sr_fin_after(c, fin, c->np_sr, gk::sr_nacc<K>() > 1));
    return GK_OK;
}

template <int K>
int sr_vec(gk_ctx *c, gk::SrArgs a, int fin) {
    const bool slabs = sr_slabs(c);
    a.fin = slabs ? gk::FIN_NONE : fin;
    {
        ProfScope ps(c, GK_KID_SR + 9 + (K == gk::SRV_BI_XS ? gk::SRV_BI_X : K));
        // the grid (hence the partial count) comes from the largest slab: the same on every rank
        gk::k_sr_vec<K, 4><<<c->np_pj, gk::TPB, 0, c->st>>>(a, c->nloc);
        LAUNCHCHK();
    }
    if (slabs) CHK(sr_fin_after(c, fin, c->np_pj, K == gk::SRV_BI_X || K == gk::SRV_BI_XS));
    return GK_OK;
}

// Two-level march (single rank; same grid as the one-level marches, so the
// partial slabs -- and every result -- are the one-level passes' bits).
template <int K2>
int sr_march2(gk_ctx *c, gk::SrArgs a, int fin) {
    a.fin = fin;
    ProfScope ps(c, GK_KID_SR + 13 + K2);
    if (c->vec == 2)
        gk::k_sr_march2<2, K2><<<c->sr_sgrid, gk::TPB, 0, c->st>>>(a);
    else
        gk::k_sr_march2<1, K2><<<c->sr_sgrid, gk::TPB, 0, c->st>>>(a);
    LAUNCHCHK();
    return GK_OK;
}

// out = M^-1 in by the generic preconditioner sweeps (Chebyshev(k)); with vdot
// the last sweep's dot <out, vdot> feeds finaliser `fin`.
int sr_prec(gk_ctx *c, const double *in, double *out, const double *vdot, int fin) {
    double *keep = c->z;
    c->z = const_cast<double *>(in);  // precond_sweeps reads its input from c->z
    const int rc = precond_sweeps(c, out, vdot != nullptr ? gk::ACC_DOT : gk::ACC_NONE, vdot, slot(c, 0));
    c->z = keep;
    CHK(rc);
    if (fin == gk::FIN_NONE) return GK_OK;
    return sr_fin_after(c, fin, c->last_np, false);
}

// One PCG iteration (cg.f90:188-232) from parity par.
int sr_pcg_iter(gk_ctx *c, int par) {
    const SrVecs v = sr_vecs(c);
    const bool id = c->pkind == GK_PREC_IDENTITY;
    gk::SrArgs a = sr_args(c);
    // p = z + beta p ; alpha = rz / <A p, p>
    a.in0 = id ? v.r : v.z;
    a.in1 = v.p[par];
    a.ou = v.p[par ^ 1];
    CHK(sr_march<gk::SRK_CG_P>(c, a, gk::FIN_CG_ALPHA));
    if (c->sr_two) {  // x += alpha p ; r -= alpha A p ; z = M^-1 r ; res, beta -- one two-level pass
        a = sr_args(c);
        a.in0 = v.p[par ^ 1];
        a.x = c->x;
        a.r = v.rr[par];
        a.oy = v.rr[par ^ 1];
        a.oz = v.z;
        return sr_march2<gk::SR2_CG_XZ>(c, a, gk::FIN_CG_RES_BETA);
    }
    // x += alpha p ; r -= alpha A p ; res = ||r|| (identity: beta = <r,r> / rz)
    a = sr_args(c);
    a.in0 = v.p[par ^ 1];
    a.x = c->x;
    a.r = v.r;
    CHK(sr_march<gk::SRK_CG_X>(c, a, id ? gk::FIN_CG_RES_ID : gk::FIN_CG_RES));
    if (id) return GK_OK;
    // z = M^-1 r ; beta = <r, z> / rz
    if (c->pkind == GK_PREC_CBPR2) {
        a = sr_args(c);
        a.in0 = v.r;
        a.oy = v.z;
        return sr_march<gk::SRK_CG_Z>(c, a, gk::FIN_CG_BETA);
    }
    return sr_prec(c, v.r, v.z, v.r, gk::FIN_CG_BETA);
}

// One BiCGSTAB iteration (bicgstab.f90:120-180) from parity par.
int sr_bicg_iter(gk_ctx *c, int par) {
    const SrVecs v = sr_vecs(c);
    const int pk = c->pkind;
    double *pn = v.p[par ^ 1], *apn = v.ap[par ^ 1];
    const double *z1 = pn, *z2 = v.s;
    // p = r + beta (p - omega ap) ; z1 = M^-1 p ; ap = A z1 ; alpha = rr0 / <ap, r0>
    gk::SrArgs a = sr_args(c);
    a.in0 = v.r;
    a.in1 = v.p[par];
    a.in2 = v.ap[par];
    a.ou = pn;
    if (c->sr_two) {  // z1 = M^-1 p, ap = A z1 and s, z2 = M^-1 s, as = A z2: two two-level passes
        a.oy = v.z1;
        a.oz = apn;
        a.vd = v.r0;
        CHK(sr_march2<gk::SR2_BI_P>(c, a, gk::FIN_BI_ALPHA));
        a = sr_args(c);
        a.in0 = v.r;
        a.in1 = apn;
        a.ou = v.s;
        a.oy = v.z2;
        a.oz = v.as;
        CHK(sr_march2<gk::SR2_BI_S>(c, a, gk::FIN_BI_OMEGA));
        z1 = v.z1;
        z2 = v.z2;
    } else if (pk == GK_PREC_IDENTITY) {
        a.oy = apn;
        a.vd = v.r0;
        CHK(sr_march<gk::SRK_BI_P>(c, a, gk::FIN_BI_ALPHA));
    } else {
        z1 = v.z1;
        z2 = v.z2;
        if (pk == GK_PREC_CBPR2) {
            a.oy = v.z1;
            CHK(sr_march<gk::SRK_BI_PC>(c, a, gk::FIN_NONE));
        } else {
            CHK(sr_vec<gk::SRV_BI_PE>(c, a, gk::FIN_NONE));
            CHK(sr_prec(c, pn, v.z1, nullptr, gk::FIN_NONE));
        }
        a = sr_args(c);
        a.in0 = v.z1;
        a.oy = apn;
        a.vd = v.r0;
        CHK(sr_march<gk::SRK_ST1>(c, a, gk::FIN_BI_ALPHA));
    }
    // s = r - alpha ap ; z2 = M^-1 s ; as = A z2 ; omega = <as, s> / <as, as>
    a = sr_args(c);
    a.in0 = v.r;
    a.in1 = apn;
    a.ou = v.s;
    if (c->sr_two) {
        // done above
    } else if (pk == GK_PREC_IDENTITY) {
        a.oy = v.as;
        CHK(sr_march<gk::SRK_BI_S>(c, a, gk::FIN_BI_OMEGA));
    } else {
        if (pk == GK_PREC_CBPR2) {
            a.oy = v.z2;
            CHK(sr_march<gk::SRK_BI_SC>(c, a, gk::FIN_NONE));
        } else {
            CHK(sr_vec<gk::SRV_BI_SE>(c, a, gk::FIN_NONE));
            CHK(sr_prec(c, v.s, v.z2, nullptr, gk::FIN_NONE));
        }
        a = sr_args(c);
        a.in0 = v.z2;
        a.oy = v.as;
        a.vd = v.s;
        CHK(sr_march<gk::SRK_ST2>(c, a, gk::FIN_BI_OMEGA));
    }
    // x = x + alpha z1 + omega z2 ; r = s - omega as ; res, beta
    a = sr_args(c);
    a.x = c->x;
    a.r = v.r;
    a.in0 = z1;
    a.in1 = z2;
    a.in2 = v.s;
    a.e0 = v.as;
    a.vd = v.r0;
    if (z2 == v.s) return sr_vec<gk::SRV_BI_XS>(c, a, gk::FIN_BI_RES);  // identity M: z2 = s
    return sr_vec<gk::SRV_BI_X>(c, a, gk::FIN_BI_RES);
}

int sr_iter(gk_ctx *c, int par) { return c->sr_solver == GK_SR_PCG ? sr_pcg_iter(c, par) : sr_bicg_iter(c, par); }

// Capture SR_GRAPH_ITERS iterations from parity 0 as one graph (single rank; a
// capture that fails leaves the eager path).
int sr_capture(gk_ctx *c) {
    HIPCHK(hipStreamBeginCapture(c->st, hipStreamCaptureModeThreadLocal));
    c->capturing = true;
    int rc = GK_OK;
    for (int i = 0; i < SR_GRAPH_ITERS && rc == GK_OK; ++i) rc = sr_iter(c, i & 1);
    c->capturing = false;
    hipGraph_t g = nullptr;
    const hipError_t e = hipStreamEndCapture(c->st, &g);
    hipGraphExec_t ge = nullptr;
    hipError_t e2 = hipErrorUnknown;
    if (rc == GK_OK && e == hipSuccess && g != nullptr) e2 = hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    if (g != nullptr) (void)hipGraphDestroy(g);
    if (rc != GK_OK || e != hipSuccess || e2 != hipSuccess) {
        (void)hipGetLastError();
        if (ge != nullptr) (void)hipGraphExecDestroy(ge);
        return set_err(GK_ERR_HIP, "capture of the short-recurrence iterations failed (%s)",
                       rc != GK_OK ? g_err.c_str() : hipGetErrorString(e != hipSuccess ? e : e2));
    }
    c->sr_graph = ge;
    return GK_OK;
}

void sr_recycle(gk_ctx *c, hipEvent_t e) { c->sr_evfree.push_back(e); }

int sr_drain(gk_ctx *c) {
    if (c->sr_pend.empty()) return GK_OK;
    const int rc = sync_st(c);
    for (hipEvent_t e : c->sr_pend) sr_recycle(c, e);
    c->sr_pend.clear();
    return rc;
}

int sr_start_body(gk_ctx *c, int solver) {
    const SrVecs v = sr_vecs(c);
    const size_t vb = sizeof(double) * (size_t)c->nloc;
    HIPCHK(hipMemsetAsync(c->x, 0, vb, c->st));
    HIPCHK(hipMemcpyAsync(v.r, c->b, vb, hipMemcpyDeviceToDevice, c->st));
    gk::SrArgs a = sr_args(c);
    if (solver == GK_SR_PCG) {
        HIPCHK(hipMemsetAsync(v.p[0], 0, vb, c->st));  // iteration 1: p = z + 0 * 0 = z  (cg.f90:183-187)
        if (c->pkind == GK_PREC_IDENTITY) {
            a.in0 = v.r;
            a.in1 = v.r;
            return sr_vec<gk::SRV_DOT>(c, a, gk::FIN_CG_INIT);
        }
        if (c->pkind == GK_PREC_CBPR2) {
            a.in0 = v.r;
            a.oy = v.z;
            return sr_march<gk::SRK_CG_Z>(c, a, gk::FIN_CG_INIT);
        }
        return sr_prec(c, v.r, v.z, v.r, gk::FIN_CG_INIT);
    }
    // r0 = p = r (bicgstab.f90:112-118); iteration 1: p = r + 0 (p - 1 * 0) = r
    HIPCHK(hipMemcpyAsync(v.r0, c->b, vb, hipMemcpyDeviceToDevice, c->st));
    HIPCHK(hipMemcpyAsync(v.p[0], c->b, vb, hipMemcpyDeviceToDevice, c->st));
    HIPCHK(hipMemsetAsync(v.ap[0], 0, vb, c->st));
    a.in0 = v.r;
    a.in1 = v.r0;
    return sr_vec<gk::SRV_DOT>(c, a, gk::FIN_BI_INIT);
}
}  // namespace

extern "C" {

int gk_sr_start(gk_ctx *c, int solver, double tol, int max_iter) {
    CHK(check_ctx(c));
    if (solver != GK_SR_PCG && solver != GK_SR_BICGSTAB) return set_err(GK_ERR_ARG, "bad solver %d", solver);
    if (max_iter < 0 || max_iter > (1 << 28)) return set_err(GK_ERR_ARG, "bad max_iter %d", max_iter);
    if (c->m < 7) return set_err(GK_ERR_ARG, "short-recurrence solvers need a context with m >= 7 (vectors)");
    HIPCHK(hipSetDevice(c->dev));
    CHK(sr_drain(c));
    c->cycle_mgs = c->cycle_hh = false;  // the Krylov columns are the solver's vectors now
    if (c->sr_dev == nullptr) {
        HIPCHK(hipMalloc(&c->sr_dev, sizeof(gk::SrDev)));
        HIPCHK(hipHostMalloc((void **)&c->sr_mir, sizeof(gk::SrMirror), hipHostMallocMapped));
        HIPCHK(hipHostGetDevicePointer((void **)&c->sr_mir_dev, c->sr_mir, 0));
    }
    if (c->sr_hist_len < std::max(max_iter, 1)) {
        if (c->sr_hist != nullptr) (void)hipFree(c->sr_hist);
        c->sr_hist = nullptr;
        c->sr_hist_len = 0;
        HIPCHK(hipMalloc(&c->sr_hist, sizeof(double) * (size_t)std::max(max_iter, 1)));
        c->sr_hist_len = std::max(max_iter, 1);
        graph_reset(c);  // a captured graph holds the old history pointer
    }
    if (c->sr_solver != solver && c->sr_graph != nullptr) {
        (void)hipGraphExecDestroy(c->sr_graph);
        c->sr_graph = nullptr;
    }
    {
        const bool two = c->tune_sr_two != 0 && c->pkind == GK_PREC_CBPR2 && !sr_slabs(c);
        if (two != c->sr_two && c->sr_graph != nullptr) {  // the captured graph runs the other passes
            (void)hipGraphExecDestroy(c->sr_graph);
            c->sr_graph = nullptr;
        }
        c->sr_two = two;
    }
    c->sr_solver = solver;
    c->sr_par = 0;
    c->sr_queued = 0;
    c->sr_maxit = max_iter;
    gk::SrDev d{};
    d.omega = 1.0;
    d.tol = tol;
    d.maxit = max_iter;
    HIPCHK(hipMemcpyAsync(c->sr_dev, &d, sizeof d, hipMemcpyHostToDevice, c->st));
    HIPCHK(hipStreamSynchronize(c->st));  // d is a stack object
    c->sr_mir->it = 0;
    c->sr_mir->done = 0;
    c->sr_mir->res = 0.0;
    return sr_start_body(c, solver);
}

int gk_sr_iterate(gk_ctx *c, int k) {
    CHK(check_ctx(c));
    if (c->sr_solver < 0) return set_err(GK_ERR_STATE, "gk_sr_iterate before gk_sr_start");
    if (k < 0 || (long long)c->sr_queued + k > c->sr_maxit)
        return set_err(GK_ERR_ARG, "gk_sr_iterate(%d): beyond max_iter %d (%d queued)", k, c->sr_maxit, c->sr_queued);
    if (k == 0) return GK_OK;
    HIPCHK(hipSetDevice(c->dev));
    const bool graphs = c->tune_graph != 0 && !collective(c) && !c->prof;
    int left = k;
    while (left > 0) {
        if (graphs && c->sr_par == 0 && left >= SR_GRAPH_ITERS) {
            if (c->sr_graph == nullptr) CHK(sr_capture(c));
            HIPCHK(hipGraphLaunch(c->sr_graph, c->st));
            left -= SR_GRAPH_ITERS;
            c->sr_queued += SR_GRAPH_ITERS;
            continue;
        }
        CHK(sr_iter(c, c->sr_par));
        c->sr_par ^= 1;
        --left;
        ++c->sr_queued;
    }
    hipEvent_t e = nullptr;
    if (!c->sr_evfree.empty()) {
        e = c->sr_evfree.back();
        c->sr_evfree.pop_back();
    } else {
        HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    HIPCHK(hipEventRecord(e, c->st));
    c->sr_pend.push_back(e);
    return GK_OK;
}

int gk_sr_status(gk_ctx *c, int wait, int *executed, int *done, double *res) {
    CHK(check_ctx(c));
    if (c->sr_solver < 0) return set_err(GK_ERR_STATE, "gk_sr_status before gk_sr_start");
    HIPCHK(hipSetDevice(c->dev));
    if (wait == 0 && !c->sr_pend.empty()) {
        hipEvent_t e = c->sr_pend.front();
        c->sr_pend.pop_front();
        const int rc = spin_until(c, query_event, e, "short-recurrence chunk");
        sr_recycle(c, e);
        CHK(rc);
        CHK(res_check(c));
        CHK(xs_check(c));
    } else {
        CHK(sr_drain(c));
        CHK(sync_st(c));
    }
    if (c->prof) CHK(prof_harvest(c));
    if (executed) *executed = __atomic_load_n(&c->sr_mir->it, __ATOMIC_ACQUIRE);
    if (done) *done = __atomic_load_n(&c->sr_mir->done, __ATOMIC_ACQUIRE);
    if (res) *res = *(volatile double *)&c->sr_mir->res;
    return GK_OK;
}

int gk_sr_history(gk_ctx *c, double *hist, int n) {
    CHK(check_ctx(c));
    if (c->sr_solver < 0) return set_err(GK_ERR_STATE, "gk_sr_history before gk_sr_start");
    if (n < 0 || n > c->sr_hist_len || hist == nullptr) return set_err(GK_ERR_ARG, "bad history length %d", n);
    HIPCHK(hipSetDevice(c->dev));
    CHK(sr_drain(c));
    if (n == 0) return GK_OK;
    HIPCHK(hipMemcpyAsync(hist, c->sr_hist, sizeof(double) * n, hipMemcpyDeviceToHost, c->st));
    return sync_st(c);
}

}  // extern "C"
