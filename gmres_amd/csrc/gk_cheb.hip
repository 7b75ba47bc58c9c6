// gk_cheb.hip -- the temporal-blocked Chebyshev(k) pass (gfx950).
// Reference: the Chebyshev(k) preconditioner is build-defined (SURVEY 8a row
// a2; README.md:11, src/preconds/chebyshev.f90:8-38 is its degree-1 cbpr2);
// each sweep is the per-sweep kernel's arithmetic, bit for bit.
#include <iterator>
#include <mutex>
#include <utility>
#include <vector>

#include "gk_cheb.hpp"

namespace gk {

// Scheduling barrier after every level (1) or only between time steps (0).
#ifndef GK_CF_LVBAR
#define GK_CF_LVBAR 0
#endif
constexpr bool CF_LVBAR = GK_CF_LVBAR != 0;

// 4c - s as ONE fma: 4c is exact (a power-of-two scale), so fma(4, c, -s)
// rounds the same real number once, exactly as (4c) - s does -- bit-identical
// to the per-sweep kernel and the oracle, one FP64 instruction per point and
// level fewer in the issue-bound level chain.  0: the multiply + subtract.
#ifndef GK_CF_FMA4
#define GK_CF_FMA4 1
#endif
__device__ __forceinline__ double cf_4c_minus(double c, double s) {
    if (GK_CF_FMA4) return __builtin_fma(4.0, c, -s);
    return 4.0 * c - s;
}


// Lane i gets lane i-1's value (lane 0 gets 0) / lane i+1's (lane 63 gets 0).
__device__ __forceinline__ double cf_from_left(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)b, 0x138, 0xF, 0xF, true);         // wave_shr:1
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), 0x138, 0xF, 0xF, true);
    return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}
__device__ __forceinline__ double cf_from_right(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)b, 0x130, 0xF, 0xF, true);         // wave_shl:1
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), 0x130, 0xF, 0xF, true);
    return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}

#ifndef GK_CF_DEPTH
#define GK_CF_DEPTH 2
#endif
constexpr int CF_U = 6;            // unroll: lcm of the 3 d slots, the 2 (res, z) slots and the ring
constexpr int CF_D = GK_CF_DEPTH;  // input lines in flight
#ifndef GK_CF_OCC
#define GK_CF_OCC 2
#endif
constexpr int CF_OCC = GK_CF_OCC;  // waves per SIMD the register budget is cut for
static_assert(CF_U % CF_D == 0, "the ring must rotate a whole number of times per unrolled trip");

template <int L, bool FIRST, bool LAST, int ACC, bool SMALL, bool STEN>
__global__ __launch_bounds__(CF_W) __attribute__((amdgpu_waves_per_eu(CF_OCC, CF_OCC))) void k_cheb_fused(CFArgs a) {
    // STEN (first pass only): the input is the Krylov column v and a stage 0
    // ahead of the levels forms the pass's z = A v row by row (the stencil
    // launch's arithmetic), so the step needs no stencil launch and no z vector
    static_assert(!STEN || (FIRST && !SMALL), "the fused stencil stage is a first-pass, full-window variant");
    constexpr int S0 = STEN ? 1 : 0;
    constexpr int LL = L + S0;                      // pipeline stages: the recompute cone and halo
    constexpr int H = cf_halo(LL);
    constexpr int D = CF_D;
    const int N = a.N;
    const int lane = threadIdx.x;
    // this window: base wb, kept points [ks, ke)
    int wb, ks, ke;
    if (SMALL || gridDim.x == 1) {
        wb = 0, ks = 0, ke = N;
    } else if (blockIdx.x == 0) {
        wb = 0, ks = 0, ke = CF_PTS - H;
    } else {
        ks = CF_PTS - H + ((int)blockIdx.x - 1) * (CF_PTS - 2 * H);
        if (blockIdx.x == gridDim.x - 1) {
            wb = N - CF_PTS, ke = N;
        } else {
            wb = ks - H, ke = ks + CF_PTS - 2 * H;
        }
    }
    const int i0 = wb + 2 * lane;           // this lane's points i0, i0+1 (even: 16-B aligned rows)
    const bool live = !SMALL || i0 < N;     // SMALL: lanes beyond the grid hold zeros
    const bool kept = i0 >= ks && i0 < ke;
    const int j0 = blockIdx.y * a.JT;
    const int j1 = min(j0 + a.JT, a.nlines);
    const bool has_lo = a.lo[0] != nullptr, has_hi = a.hi[0] != nullptr;
    double acc = 0.0;
    // FAST steps load the slab vectors through buffer descriptors: the row
    // offset is a scalar, the lane's column offset one 32-bit VGPR (no 64-bit
    // address registers per stream; the host keeps slabs below 2 GiB)
    const int rowb = N * 8, voff = i0 * 8, nbytes = a.nlines * rowb;
    auto rsrc = [&](const double *p) {
        return __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(p), (short)0, nbytes, 0x00020000);
    };
    const auto rs_din = rsrc(a.din), rs_vdot = rsrc(a.vdot);
    const auto rs_rin = rsrc(FIRST ? a.din : a.rin), rs_zin = rsrc(FIRST ? a.din : a.zin);
    auto bload = [&](__amdgpu_buffer_rsrc_t r, int so) {
        return __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(r, voff, so, 0));
    };
    // Stores stay global_store: a 16-byte buffer_store with an SGPR soffset was
    // emitted with NO wait state before the next VALU overwrote its data VGPRs
    // (the hazard recogniser exempts SGPR-soffset MUBUF stores), and on gfx950
    // such stores wrote corrupted values at random rows (measured: the fused
    // reductions' variants, where the reduction reuses the stored registers).

    // level state: d[l][slot][point] and res[l][slot][point] in registers; the
    // running sum z of each level in LDS, zs[l][lane] = z of the line level l
    // computes next.  Every lane touches only its own element (no barrier), and
    // a level reads its z before the level above overwrites it with the new
    // line's (a wave's LDS operations complete in order).
    double d[L][3][2], r[L][2][2];
    double vw[3][2];  // STEN: three lines of v
    __shared__ double2 zs[L][CF_W];
#pragma unroll
    for (int q = 0; q < 3; ++q) vw[q][0] = vw[q][1] = 0.0;
#pragma unroll
    for (int l = 0; l < L; ++l) {
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            d[l][0][k] = d[l][1][k] = d[l][2][k] = 0.0;
            r[l][0][k] = r[l][1][k] = 0.0;
        }
        zs[l][lane] = double2{0.0, 0.0};
    }
    // the ring: input lines t+1..t+D, and the dot partners of the lines the
    // last level emits
    double pd[D][2], pr[D][2], pz[D][2];
    double2 pv[D];
#pragma unroll
    for (int s = 0; s < D; ++s) pv[s] = double2{0.0, 0.0};

    auto ld2 = [&](int which, const double *base, int row, double (&v)[2]) {
        v[0] = v[1] = 0.0;
        const double *p;
        if (row < 0) {
            if (!has_lo || row < -LL) return;
            p = a.lo[which] + (i64)(row + LL) * N + i0;
        } else if (row >= a.nlines) {
            if (!has_hi || row >= a.nlines + LL) return;
            p = a.hi[which] + (i64)(row - a.nlines) * N + i0;
        } else {
            p = base + (i64)row * N + i0;
        }
        if (live) {
            const double2 t = *reinterpret_cast<const double2 *>(p);
            v[0] = t.x;
            v[1] = t.y;
        }
    };
    auto issue_in = [&](bool fast, int row, int s) {
        if (fast) {
            const int so = row * rowb;
            const double2 t = bload(rs_din, so);
            pd[s][0] = t.x;
            pd[s][1] = t.y;
            if (!FIRST) {
                const double2 u = bload(rs_rin, so), w = bload(rs_zin, so);
                pr[s][0] = u.x, pr[s][1] = u.y, pz[s][0] = w.x, pz[s][1] = w.y;
            }
        } else {
            ld2(0, a.din, row, pd[s]);
            if (!FIRST) {
                ld2(1, a.rin, row, pr[s]);
                ld2(2, a.zin, row, pz[s]);
            }
        }
    };
    auto issue_dot = [&](bool fast, int row, int s) {
        if (!(LAST && ACC == ACC_DOT)) return;
        if (fast) {
            pv[s] = bload(rs_vdot, row * rowb);
        } else if (row >= j0 && row < j1 && kept) {
            pv[s] = *reinterpret_cast<const double2 *>(a.vdot + (i64)row * N + i0);
        }
    };
    const int tb0 = j0 - LL, tend = j1 + LL;

    // One time step t (phase U of the unrolled trip).  FAST: every level
    // computes a row inside the grid (or a neighbour's halo) that reaches the
    // kept rows, and the ring refills from slab rows -- no tests at all.
    auto step = [&](auto fastc, auto uc, int t) {
        constexpr bool FAST = decltype(fastc)::value;
        constexpr int U = decltype(uc)::value;
        constexpr int SS = U % 3, SC = (U + 1) % 3, SN = (U + 2) % 3;  // d slots: rows R-2, R-1, R
        constexpr int QC = (U + 1) % 2, QN = U % 2;                     // (res, z) slots: R-1, R
        constexpr int RS = U % D;                                       // ring slot of line t
        // level -1 emits the input line t into level 0's incoming slots (STEN:
        // stage 0 takes line t of v and emits z = A v of line t - 1)
        if (STEN) {
            vw[SN][0] = pd[RS][0];
            vw[SN][1] = pd[RS][1];
            const int srow = t - 1;
            bool zero = false, run = true;
            if (!FAST) {
                zero = (!has_lo && srow < 0) || (!has_hi && srow >= a.nlines);
                run = !zero && srow >= j0 - L && srow < j1 + L;
            }
            // values first, then unconditional stores into the state (stores in
            // the branches get merged through a pointer phi, which keeps the
            // state arrays out of registers)
            double nd0 = d[0][SN][0], nd1 = d[0][SN][1], nr0 = r[0][QN][0], nr1 = r[0][QN][1];
            if (zero) {
                nd0 = nd1 = 0.0;
            } else if (run) {
                const double C0 = vw[SC][0], C1 = vw[SC][1];
                const double W0 = cf_from_left(C1), E1 = cf_from_right(C0);
                const double s0 = ((W0 + C1) + vw[SN][0]) + vw[SS][0];
                const double s1 = ((C0 + E1) + vw[SN][1]) + vw[SS][1];
                const double ax0 = cf_4c_minus(C0, s0), ax1 = cf_4c_minus(C1, s1);
                nd0 = ax0 / a.theta;
                nd1 = ax1 / a.theta;
                nr0 = ax0;
                nr1 = ax1;
            }
            d[0][SN][0] = nd0, d[0][SN][1] = nd1, r[0][QN][0] = nr0, r[0][QN][1] = nr1;
        } else {
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                if (FIRST) {
                    d[0][SN][k] = pd[RS][k] / a.theta;
                    r[0][QN][k] = pd[RS][k];
                } else {
                    d[0][SN][k] = pd[RS][k];
                    r[0][QN][k] = pr[RS][k];
                }
            }
        }
        // z of the line level 0 computes now; then the input line's z takes its place
        double2 zcur = double2{0.0, 0.0};
        if (!FIRST) {
            zcur = zs[0][lane];
            zs[0][lane] = double2{pz[RS][0], pz[RS][1]};
        }
        if (FAST || t + D < tend) issue_in(FAST, t + D, RS);
        double od[2] = {0.0, 0.0}, orr[2] = {0.0, 0.0}, oz[2] = {0.0, 0.0};  // the last level's emission
#pragma unroll
        for (int l = 0; l < L; ++l) {
            const int row = t - l - 1 - S0;  // the row level l computes
            // read ahead the z level l+1 consumes in this step, before this level
            // writes the z of its new line in its place
            const double2 znext = (l + 1 < L) ? zs[l + 1][lane] : double2{0.0, 0.0};
            bool zero = false, run = true;
            if (!FAST) {
                zero = (!has_lo && row < 0) || (!has_hi && row >= a.nlines);
                run = !zero && row >= j0 - (L - 1 - l) && row < j1 + (L - 1 - l);
            }
            if (zero) {
                if (l + 1 < L) {
                    d[l + 1][SN][0] = d[l + 1][SN][1] = 0.0;
                } else {
                    od[0] = od[1] = 0.0;
                }
            } else if (run) {
                const double C0 = d[l][SC][0], C1 = d[l][SC][1];
                const double W0 = cf_from_left(C1), E1 = cf_from_right(C0);
                const double s0 = ((W0 + C1) + d[l][SN][0]) + d[l][SS][0];
                const double s1 = ((C0 + E1) + d[l][SN][1]) + d[l][SS][1];
                const double ad0 = cf_4c_minus(C0, s0), ad1 = cf_4c_minus(C1, s1);
                const double res0 = r[l][QC][0] - ad0, res1 = r[l][QC][1] - ad1;
                double dn0 = a.c1[l] * C0 + a.c2[l] * res0, dn1 = a.c1[l] * C1 + a.c2[l] * res1;
                // z of level 0 in the first pass equals its d (z0 = d0)
                const double zc0 = (FIRST && l == 0) ? C0 : zcur.x;
                const double zc1 = (FIRST && l == 0) ? C1 : zcur.y;
                double zn0 = zc0 + dn0, zn1 = zc1 + dn1;
                double rn0 = res0, rn1 = res1;
                if (SMALL && !live) dn0 = dn1 = rn0 = rn1 = zn0 = zn1 = 0.0;
                if (l + 1 < L) {
                    d[l + 1][SN][0] = dn0, d[l + 1][SN][1] = dn1;
                    r[l + 1][QN][0] = rn0, r[l + 1][QN][1] = rn1;
                    zs[l + 1][lane] = double2{zn0, zn1};
                } else {
                    od[0] = dn0, od[1] = dn1, orr[0] = rn0, orr[1] = rn1, oz[0] = zn0, oz[1] = zn1;
                }
            }
            zcur = znext;
            if (CF_LVBAR) __builtin_amdgcn_sched_barrier(0);
        }
        // the last level emitted row t - LL
        const int orow = t - LL;
        if ((FAST || (orow >= j0 && orow < j1)) && kept) {
            const i64 idx = (i64)orow * N + i0;
            if (LAST) {
                *reinterpret_cast<double2 *>(a.out + idx) = double2{oz[0], oz[1]};
                if (ACC == ACC_DOT) {
                    acc = acc + oz[0] * pv[RS].x;
                    acc = acc + oz[1] * pv[RS].y;
                } else if (ACC == ACC_NORM) {
                    acc = acc + oz[0] * oz[0];
                    acc = acc + oz[1] * oz[1];
                }
            } else {
                *reinterpret_cast<double2 *>(a.dout + idx) = double2{od[0], od[1]};
                *reinterpret_cast<double2 *>(a.rout + idx) = double2{orr[0], orr[1]};
                *reinterpret_cast<double2 *>(a.zout + idx) = double2{oz[0], oz[1]};
            }
        }
        // the partner of the row emitted D steps from now
        if (FAST || t + D < tend) issue_dot(FAST, t + D - LL, RS);
        // keep the scheduler from hoisting the next step's work over this one
        // (only the 4 doubles per point and level above are live across it)
        __builtin_amdgcn_sched_barrier(0);
    };
    using F = std::false_type;
    using T = std::true_type;
    auto trip = [&](auto fastc, int tb, int tz) {
        step(fastc, std::integral_constant<int, 0>{}, tb);
        if (decltype(fastc)::value || tb + 1 < tz) step(fastc, std::integral_constant<int, 1>{}, tb + 1);
        if (decltype(fastc)::value || tb + 2 < tz) step(fastc, std::integral_constant<int, 2>{}, tb + 2);
        if (decltype(fastc)::value || tb + 3 < tz) step(fastc, std::integral_constant<int, 3>{}, tb + 3);
        if (decltype(fastc)::value || tb + 4 < tz) step(fastc, std::integral_constant<int, 4>{}, tb + 4);
        if (decltype(fastc)::value || tb + 5 < tz) step(fastc, std::integral_constant<int, 5>{}, tb + 5);
    };
    if (j0 < a.nlines) {
#pragma unroll
        for (int s = 0; s < D; ++s) {
            issue_in(false, tb0 + s, s);
            issue_dot(false, tb0 + s - LL, s);
        }
        // FAST steps: t >= j0 + LL (every stage's row reaches the kept rows),
        // rows t-LL..t-1 inside the grid unless a neighbour's halo covers them,
        // ring refills t + D inside the slab.  Segment boundaries are whole
        // trips from tb0, so every ring / state slot stays compile-time.
        const int lo = j0 + LL;
        const int hi = min(min(tend, a.nlines - D), has_hi ? tend : a.nlines + 1);
        int tf0 = tend, tf1 = tend;
        const int f0 = tb0 + (max(lo, tb0) - tb0 + CF_U - 1) / CF_U * CF_U;
        // (SMALL: never -- a FAST load would read past the row into dead lanes)
        const int nf = (!SMALL && hi > f0) ? (hi - f0) / CF_U : 0;
        if (nf > 0) {
            tf0 = f0;
            tf1 = f0 + nf * CF_U;
        }
        for (int tb = tb0; tb < tf0; tb += CF_U) trip(F{}, tb, tf0);
        // Drain once before the FAST loop: its header is the first use of the
        // ring slot loaded D steps earlier, and entering from the prologue with
        // that slot's load the most recent one made the compiler wait for ALL
        // loads there on every trip (vmcnt(0) once per 6 steps: the ring's
        // prefetch lost); with nothing outstanding on entry only the loop's own
        // back edge counts and the header waits for the one slot it needs.
        __builtin_amdgcn_s_waitcnt(0);
        for (int tb = tf0; tb < tf1; tb += CF_U) trip(T{}, tb, tf1);
        for (int tb = tf1; tb < tend; tb += CF_U) trip(F{}, tb, tend);
    }
    if (ACC != ACC_NONE) {
        const double s = wave_sum(acc);
        if (lane == 0) a.part[(i64)blockIdx.y * gridDim.x + blockIdx.x] = s;
    }
}

#ifndef GK_CF_JT
#define GK_CF_JT 0  // 0: JT chosen per pass; any other value: that JT (A/B builds)
#endif

namespace {

// Workgroups per CU, queried once per (kernel, device): every Arnoldi step
// launches a pass.  0: the build spilled this kernel's registers to scratch
// -- refused, because a build whose FAST steps mixed buffer loads with scratch
// reloads gave wrong results once a workgroup ran more than two unrolled trips
// (measured at 2048^2 and 4096^2 while 1024^2 was bit-exact).
template <typename K>
int occupancy(K kern, int dev) {
    static std::mutex mu;
    static std::vector<std::pair<std::pair<const void *, int>, int>> seen;
    std::lock_guard<std::mutex> lk(mu);
    const auto key = std::make_pair(reinterpret_cast<const void *>(kern), dev);
    for (const auto &e : seen)
        if (e.first == key) return e.second;
    int occ = 0;
    hipFuncAttributes fa{};
    if (hipFuncGetAttributes(&fa, reinterpret_cast<const void *>(kern)) == hipSuccess && fa.localSizeBytes > 0) {
        occ = 0;
    } else if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern, CF_W, 0) != hipSuccess || occ <= 0) {
        occ = 8;
    }
    seen.emplace_back(key, occ);
    return occ;
}

// A workgroup marches JT + 2L time steps (the recompute cone), so JT
// minimises  rounds x (JT + 2L)  where a round is one wave of resident
// workgroups (occupancy x CUs): at 4096^2, L = 8 (2 waves per SIMD) JT = 80
// gives 1924 workgroups in ONE round where 64 would need two.
// GK_CF_JTFINE (default): every even JT from 16 to 256 is a candidate, so the
// one round fills the resident slots as tightly as the window count allows
// (4096^2, L = 8: JT = 78, 2014 workgroups of 96 steps, where 80 gave 1976 of 98).
#ifndef GK_CF_JTFINE
#define GK_CF_JTFINE 1
#endif
int pick_jt(int gx, int lines, int L, i64 cap) {
    static const int jts_coarse[] = {16, 24, 32, 48, 64, 80, 96, 128, 160, 192, 256, 384, 512, 1024, 2048, 4096, 8192};
    static const std::vector<int> jts_fine = [] {
        std::vector<int> v;
        for (int jt = 16; jt <= 256; jt += 2) v.push_back(jt);
        for (int jt : {384, 512, 1024, 2048, 4096, 8192}) v.push_back(jt);
        return v;
    }();
    const std::vector<int> jts = GK_CF_JTFINE ? jts_fine : std::vector<int>(std::begin(jts_coarse), std::end(jts_coarse));
    i64 best = -1;
    int JT = GK_CF_JT > 0 ? GK_CF_JT : 64;
    for (int jt : jts) {
        if (GK_CF_JT > 0 && jt != GK_CF_JT) continue;
        const i64 nb = (i64)gx * ((lines + jt - 1) / jt);
        if (nb > NPMAX) continue;
        const i64 cost = ((nb + cap - 1) / cap) * (jt + 2 * L);
        if (best < 0 || cost < best) {
            best = cost;
            JT = jt;
        }
        if (jt >= lines) break;
    }
    // No candidate kept the partial count within a reduction slot (a fixed-JT
    // A/B build, or a very wide grid): grow JT until it does -- a larger grid
    // would write past its slot into the next one.
    while (best < 0 && (i64)gx * ((lines + JT - 1) / JT) > NPMAX && JT < lines) JT *= 2;
    return JT;
}

template <int L, bool FIRST, bool LAST, int ACC, bool SMALL, bool STEN = false>
int launch(const CFLaunch &q, CFArgs &a, i64 *np) {
    auto kern = k_cheb_fused<L, FIRST, LAST, ACC, SMALL, STEN>;
    const int gx = cf_windows(a.N, L + (STEN ? 1 : 0));
    const int occ = occupancy(kern, q.dev);
    if (occ == 0) return GK_CF_ESPILL;
    const i64 cap = (i64)occ * (q.cus > 0 ? q.cus : 256);
    const int JT = pick_jt(gx, q.lines, L + (STEN ? 1 : 0), cap);
    const dim3 g(gx, (q.lines + JT - 1) / JT, 1);
    if (ACC != ACC_NONE && (i64)g.x * g.y > NPMAX) return GK_CF_ESLOT;
    a.JT = JT;
    kern<<<g, CF_W, 0, q.st>>>(a);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
    if (np != nullptr) *np = (i64)g.x * g.y;
    return 0;
}

}  // namespace

// One pass of L sweeps with the fused reduction q.acc; grids narrower than one
// window run the SMALL variant.  Instantiated per L in one of GK_CF_PARTS
// translation units (the unrolled kernels dominate the build time).
template <int L, bool FIRST, bool LAST>
int cf_launch_acc(const CFLaunch &q, CFArgs &a, i64 *np) {
    if constexpr (FIRST && LAST) {
        if (q.sten) {  // the Arnoldi step's pass with its stencil: ACC_DOT, full windows only
            if (q.acc != ACC_DOT || a.N < CF_PTS) return GK_CF_ESTEN;
            return launch<L, true, true, ACC_DOT, false, true>(q, a, np);
        }
    }
    const bool small = a.N < CF_PTS;
    if (q.acc == ACC_DOT)
        return small ? launch<L, FIRST, LAST, ACC_DOT, true>(q, a, np) : launch<L, FIRST, LAST, ACC_DOT, false>(q, a, np);
    if (q.acc == ACC_NORM)
        return small ? launch<L, FIRST, LAST, ACC_NORM, true>(q, a, np)
                     : launch<L, FIRST, LAST, ACC_NORM, false>(q, a, np);
    return small ? launch<L, FIRST, LAST, ACC_NONE, true>(q, a, np) : launch<L, FIRST, LAST, ACC_NONE, false>(q, a, np);
}

// The first of two passes: always CF_LMAX sweeps, no reduction.
int cf_launch_first(const CFLaunch &q, CFArgs &a, i64 *np);

// Which translation unit instantiates the passes of L levels: parts balanced
// by unrolled size (8 + 1, 7 + 2, 6 + 3, 5 + 4; the dispatcher in part 0).
// GK_CF_PART unset: one translation unit holds everything (A/B builds).
#define GK_CF_DECL(L, EXT)                                                       \
    EXT template int cf_launch_acc<L, true, true>(const CFLaunch &, CFArgs &, i64 *); \
    EXT template int cf_launch_acc<L, false, true>(const CFLaunch &, CFArgs &, i64 *);
#ifdef GK_CF_PART
#define GK_CF_MINE(L) (GK_CF_PART == ((L) >= 5 ? 8 - (L) : (L) - 1))
#else
#define GK_CF_MINE(L) 1
#endif
#if GK_CF_MINE(1)
GK_CF_DECL(1, )
#endif
#if GK_CF_MINE(2)
GK_CF_DECL(2, )
#endif
#if GK_CF_MINE(3)
GK_CF_DECL(3, )
#endif
#if GK_CF_MINE(4)
GK_CF_DECL(4, )
#endif
#if GK_CF_MINE(5)
GK_CF_DECL(5, )
#endif
#if GK_CF_MINE(6)
GK_CF_DECL(6, )
#endif
#if GK_CF_MINE(7)
GK_CF_DECL(7, )
#endif
#if GK_CF_MINE(8)
GK_CF_DECL(8, )
int cf_launch_first(const CFLaunch &q, CFArgs &a, i64 *np) {
    return a.N < CF_PTS ? launch<CF_LMAX, true, false, ACC_NONE, true>(q, a, np)
                        : launch<CF_LMAX, true, false, ACC_NONE, false>(q, a, np);
}
#endif

#if !defined(GK_CF_PART) || GK_CF_PART == 0
#ifdef GK_CF_PART
GK_CF_DECL(2, extern)
GK_CF_DECL(3, extern)
GK_CF_DECL(4, extern)
GK_CF_DECL(5, extern)
GK_CF_DECL(6, extern)
GK_CF_DECL(7, extern)
#endif

template <bool FIRST, bool LAST>
int launch_l(const CFLaunch &q, CFArgs &a, i64 *np) {
    switch (q.L) {
        case 1: return cf_launch_acc<1, FIRST, LAST>(q, a, np);
        case 2: return cf_launch_acc<2, FIRST, LAST>(q, a, np);
        case 3: return cf_launch_acc<3, FIRST, LAST>(q, a, np);
        case 4: return cf_launch_acc<4, FIRST, LAST>(q, a, np);
        case 5: return cf_launch_acc<5, FIRST, LAST>(q, a, np);
        case 6: return cf_launch_acc<6, FIRST, LAST>(q, a, np);
        case 7: return cf_launch_acc<7, FIRST, LAST>(q, a, np);
        default: return cf_launch_acc<8, FIRST, LAST>(q, a, np);
    }
}

// The passes a degree k <= 2 CF_LMAX needs: (FIRST, LAST) for k <= 8, else
// (FIRST, !LAST) of 8 sweeps then (!FIRST, LAST) of the rest.
int cheb_launch(const CFLaunch &q, CFArgs &a, i64 *np) {
    if (q.first && q.last) return launch_l<true, true>(q, a, np);
    if (q.first) return cf_launch_first(q, a, np);
    return launch_l<false, true>(q, a, np);
}
#endif

}  // namespace gk
