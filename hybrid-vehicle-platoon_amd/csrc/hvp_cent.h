// hvp_cent.h -- the centralised platoon QP (MpcMldCent, mpcs/cent_mld.py:21-182) for a GIVEN
// (possibly partial) region assignment, solved by ONE 64-lane wavefront.
//
// MpcMldCent builds one MIQP over the whole platoon: the n vehicles' MLD models (MpcMldCentDecup
// [EXT], constrain_first_state=False), leader tracking of x_ref (:85-105), chain spacing terms
// |x_i - x_{i-1} - spacing(x_i)|^2_Q (:106-117), Q_u u^2 and Q_du (du)^2 per vehicle (:119-135), the
// slack cost w s (:137-140), the acceleration rows (:145-163) and the soft safe distance
// p_i <= p_{i-1} - d_safe + s_i (:170-177; plus the leader's row w.r.t. x_ref with
// real_vehicle_as_reference, :164-169).  With every vehicle's region sequence fixed it is a convex
// QP in the n N velocities y_{i,a} = v_{i,a+1} -- the decentralised condensed QP of every vehicle
// (hvp_gi.h) plus the chain coupling:
//   * the chain term couples consecutive vehicles through constant 2x2 blocks (pure weights),
//     so the Hessian is block tridiagonal with closed-form blocks (no per-step data);
//   * the soft safe-distance row of follower i at step k involves both prefixes:
//     ts (sum_{b<k-1} y_{i,b} - sum_{b<k-1} y_{i-1,b}) <= -d_safe - (P1_i - P1_{i-1}).
//
// Lane t = i N + a owns variable y_{i,a} and the rows of state k = a + 1 of vehicle i: V, U, A
// (as hvp_gi.h), P_lo / P_hi on p_{i,a+1} and the soft SF row (a >= 1).  J and R (V x V,
// V = n N <= 64) live in dynamic LDS with row stride V + 1 doubles; the Goldfarb-Idnani iteration
// is that of hvp_coop.h with wave-wide (width 64) shuffles and a row normal given by at most two
// contiguous segments of lanes.  Vehicle i's steps a >= K_i are relaxed (branch and bound,
// hvp_cent_bnb.h).
#pragma once

#include <hip/hip_runtime.h>

#include "hvp_bnb.h"
#include "hvp_gi.h"
#include "hvp_ipm.h"

namespace hvp {
namespace cent {

constexpr int W = 64;
constexpr int kMaxV = 64;     // one lane per velocity variable
constexpr int kMaxVeh = 16;
constexpr int ROWS = 9;       // rows per lane
constexpr int REV = 1 << 10;  // reversed copy of a saturated soft row

// LDS carve of one wave: J, R (V x (V+1), row stride V + 1), a 64-entry vector and the
// min_1_norm LP's row-descriptor buffer (64 rows x 10 doubles, hvp_cent_l1.h)
struct Lds {
    double* J;
    double* R;
    double* v;
    double* desc;
    int LD;
};
HVP_HD inline size_t lds_doubles(int V, bool l1 = false) { return (size_t)2 * V * (V + 1) + W + (l1 ? W * 10 : 0); }
__device__ inline Lds lds_carve(double* base, int V) {
    Lds s;
    s.LD = V + 1;
    s.J = base;
    s.R = base + (size_t)V * (V + 1);
    s.v = s.R + (size_t)V * (V + 1);
    s.desc = s.v + W;
    return s;
}

__device__ inline int lane() { return (int)(threadIdx.x & (W - 1)); }
__device__ inline void wsync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
}

// ---- cross-lane primitives.  A generic __shfl is a ds_bpermute round trip through the LDS
// crossbar (~100+ cycles); the solver's chains of broadcasts and reductions use instead
//   * v_readlane (SGPR result) for a broadcast from a wave-uniform source lane (bcu), and
//   * DPP (quad_perm, row mirrors, row_shr) inside 16-lane rows plus readlanes across rows.
// bc() (ds_bpermute) remains for lane-varying sources.
template <class T>
__device__ inline T bc(T x, int src) { return __shfl(x, src, W); }
__device__ inline int bcu(int x, int src) { return __builtin_amdgcn_readlane(x, src); }
__device__ inline double bcu(double x, int src) {
    const long long b = __double_as_longlong(x);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)b, src);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(b >> 32), src);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
__device__ inline uint64_t bcu(uint64_t x, int src) {
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)x, src);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(x >> 32), src);
    return ((uint64_t)hi << 32) | lo;
}
constexpr int kDppXor1 = 0xB1;        // quad_perm [1,0,3,2]
constexpr int kDppXor2 = 0x4E;        // quad_perm [2,3,0,1]
constexpr int kDppHalfMirror = 0x141; // row_half_mirror
constexpr int kDppMirror = 0x140;     // row_mirror
template <int CTRL>
__device__ inline int dppi(int x) { return __builtin_amdgcn_mov_dpp(x, CTRL, 0xf, 0xf, false); }
template <int CTRL>
__device__ inline double dppd(double x) {
    const long long b = __double_as_longlong(x);
    const unsigned lo = (unsigned)__builtin_amdgcn_mov_dpp((int)b, CTRL, 0xf, 0xf, false);
    const unsigned hi = (unsigned)__builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xf, 0xf, false);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
// row_shr:k with zero fill of the lanes without a source
template <int K>
__device__ inline double dpp_shr0(double x) {
    const long long b = __double_as_longlong(x);
    const unsigned lo = (unsigned)__builtin_amdgcn_update_dpp(0, (int)b, 0x110 + K, 0xf, 0xf, true);
    const unsigned hi = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(b >> 32), 0x110 + K, 0xf, 0xf, true);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
// sum over the wave, identical in every lane
__device__ inline double wsum(double x) {
    x += dppd<kDppXor1>(x);
    x += dppd<kDppXor2>(x);
    x += dppd<kDppHalfMirror>(x);
    x += dppd<kDppMirror>(x);
    return (bcu(x, 0) + bcu(x, 16)) + (bcu(x, 32) + bcu(x, 48));
}
__device__ inline int wor(int x) { return __ballot(x != 0) != 0ull ? 1 : 0; }
__device__ inline double wmax(double x) {
    x = fmax(x, dppd<kDppXor1>(x));
    x = fmax(x, dppd<kDppXor2>(x));
    x = fmax(x, dppd<kDppHalfMirror>(x));
    x = fmax(x, dppd<kDppMirror>(x));
    return fmax(fmax(bcu(x, 0), bcu(x, 16)), fmax(bcu(x, 32), bcu(x, 48)));
}
// inclusive prefix sum over the wave (row-local Hillis-Steele, then the row carries)
__device__ inline double wscan(double x) {
    const int t = lane();
    x += dpp_shr0<1>(x);
    x += dpp_shr0<2>(x);
    x += dpp_shr0<4>(x);
    x += dpp_shr0<8>(x);
    const double r0 = bcu(x, 15), r1 = bcu(x, 31), r2 = bcu(x, 47);
    const int row = t >> 4;
    return x + (row == 0 ? 0.0 : (row == 1 ? r0 : (row == 2 ? r0 + r1 : (r0 + r1) + r2)));
}
// x of lane t - 1 (lane 0: 0)
__device__ inline double shift_up1(double x) {
    const int t = lane();
    const double y = dpp_shr0<1>(x);
    const double c15 = bcu(x, 15), c31 = bcu(x, 31), c47 = bcu(x, 47);
    return t == 16 ? c15 : (t == 32 ? c31 : (t == 48 ? c47 : y));
}
// (key, who) minimum with ties to the lower index, identical in every lane
__device__ inline void wargmin(double& key, int& who) {
    auto step = [&](double ok, int ow) {
        if (ok < key || (ok == key && ow < who)) {
            key = ok;
            who = ow;
        }
    };
    step(dppd<kDppXor1>(key), dppi<kDppXor1>(who));
    step(dppd<kDppXor2>(key), dppi<kDppXor2>(who));
    step(dppd<kDppHalfMirror>(key), dppi<kDppHalfMirror>(who));
    step(dppd<kDppMirror>(key), dppi<kDppMirror>(who));
    double bk = bcu(key, 0);
    int bw = bcu(who, 0);
#pragma unroll
    for (int r = 16; r < W; r += 16) {
        const double k2 = bcu(key, r);
        const int w2 = bcu(who, r);
        if (k2 < bk || (k2 == bk && w2 < bw)) {
            bk = k2;
            bw = w2;
        }
    }
    key = bk;
    who = bw;
}

// HVP_CENT_DEBUG >= 3: shader-clock cycles per phase of the wave QP, summed over the launch
// (0 setup, 1 Cholesky, 2 minimiser + J, 3 most-violated search, 4 dv / z, 5 r back-substitution,
// 6 step lengths, 7 add, 8 drop, 9 direct cost, 10 QPs, 11 iterations)
__device__ unsigned long long g_cent_prof[16];
#ifdef HVP_CENT_PROF
struct Prof {
    bool on;
    long long last;
    unsigned long long acc[12];
    __device__ void start(bool enable) {
        on = enable;
        for (int k = 0; k < 12; ++k) acc[k] = 0;
        last = on ? clock64() : 0;
    }
    __device__ void mark(int k) {
        if (!on) return;
        const long long now = clock64();
        acc[k] += (unsigned long long)(now - last);
        last = now;
    }
    __device__ void count(int k) {
        if (on) acc[k] += 1;
    }
    __device__ void flush() {
        if (!on || (threadIdx.x & 63) != 0) return;
        for (int k = 0; k < 12; ++k) atomicAdd(&g_cent_prof[k], acc[k]);
    }
};
#else  // profiling compiled out (make PROF=1 builds it in)
struct Prof {
    __device__ void start(bool) {}
    __device__ void mark(int) {}
    __device__ void count(int) {}
    __device__ void flush() {}
};
#endif

// One platoon instance: n vehicles, horizon N, leader index / spacing flag, per-vehicle systems.
struct Inst {
    int n, N, V, L;
    bool lsp;                   // real_vehicle_as_reference: leader spacing term and its safe row
    const hvp_system* systems;  // the handle's table
    const int32_t* vsys;        // [n] system index per vehicle
    const double* x0;           // [2n] (p0, v0) per vehicle
    const double* xl;           // leader_x (2, N+1)
    int debug;                  // HVP_CENT_DEBUG: printf diagnostics of failing QPs
};

struct Lane {
    int i, a;
    bool on;
    double v0, P1, ts, pmin, pmax;
    double am, vlo, vhi, ulo, uhi, dec, acc;
    double ub, uc;  // input map of step a: u = (v_{a+1} - am v_a - uc) / ub
    bool ucost;     // step a carries its input cost (fixed, or relaxed in a virtual region)
    int sf;       // 0 none, 1 pair row with vehicle i-1, 2 leader row w.r.t. x_ref
    double sfd;   // SF row: s_i(y) <= sfd with s = p_{i,a+1} (- p_{i-1,a+1})  (constants folded)
    double y, f;
};

// exclusive prefix sum of y over the lanes of the same vehicle (cum_{i,a} = sum_{b<a} y_{i,b})
__device__ inline double vehicle_prefix(double y, int N) {
    const int t = lane();
    const double inc = wscan(y);
    const int s0 = (t / N) * N;
    const double base = __shfl(inc, s0 > 0 ? s0 - 1 : 0, W);
    return inc - y - (s0 > 0 ? base : 0.0);
}

// chain / leader quadratic forms (constant weights): self block of vehicle i, linear part per step
struct Forms {
    double Wpp, Wpv, Wvv;          // self block of vehicle i (per step k = 1..N)
    double Cpp, Cpv, Cvp, Cvv;     // coupling of (i, i-1): 2 (Cpp p_i p_j + Cpv p_i v_j + Cvp v_i p_j + Cvv v_i v_j)
};

__device__ inline Forms forms(const Consts& C, const Inst& I, int i) {
    const double qpp = C.Qpp, qpv = C.Qpv, qvv = C.Qvv, t0 = C.t0;
    Forms F{0, 0, 0, 0, 0, 0, 0};
    if (i == I.L) {  // |x - x_ref (- spacing(x))|^2_Q
        const double tl = I.lsp ? t0 : 0.0;
        F.Wpp += qpp;
        F.Wpv += qpp * tl + qpv;
        F.Wvv += qpp * tl * tl + 2.0 * qpv * tl + qvv;
    }
    if (i >= 1) {  // follower of the pair (i, i-1): e = (p_i + t0 v_i + d0 - p_{i-1}, v_i - v_{i-1})
        F.Wpp += qpp;
        F.Wpv += qpp * t0 + qpv;
        F.Wvv += qpp * t0 * t0 + 2.0 * qpv * t0 + qvv;
    }
    if (i + 1 < I.n) {  // predecessor in the pair (i+1, i)
        F.Wpp += qpp;
        F.Wpv += qpv;
        F.Wvv += qvv;
    }
    F.Cpp = -qpp;
    F.Cpv = -qpv;
    F.Cvp = -(qpp * t0 + qpv);
    F.Cvv = -(qpv * t0 + qvv);
    return F;
}

// linear part (x'Wx + 2 l'x convention) of vehicle i's own terms at step k (data: x_ref, d0)
__device__ inline void lin(const Consts& C, const Inst& I, int i, int k, double& lp, double& lv) {
    const double qpp = C.Qpp, qpv = C.Qpv, qvv = C.Qvv, t0 = C.t0, d0 = C.d0;
    lp = 0.0;
    lv = 0.0;
    if (i == I.L) {
        const double tl = I.lsp ? t0 : 0.0;
        const double r0 = -I.xl[k] + (I.lsp ? d0 : 0.0), r1 = -I.xl[I.N + 1 + k];
        const double a0 = qpp * r0 + qpv * r1, a1 = qpv * r0 + qvv * r1;
        lp += a0;
        lv += tl * a0 + a1;
    }
    if (i >= 1) {
        lp += d0 * qpp;
        lv += d0 * (qpp * t0 + qpv);
    }
    if (i + 1 < I.n) {
        lp -= d0 * qpp;
        lv -= d0 * qpv;
    }
}

// Lane data and Hessian row t (into LDS J) for the assignment ci (region code of the lane's
// vehicle) with Ki fixed steps of that vehicle; [lo, hi] is the exact interval of v_{Ki} of the
// lane's vehicle, from which the undecided steps are relaxed (hvp_ipm.h:relax_step, the oracle's
// relax_tail).  Returns false if a constant row is violated (p_1 outside the position box).
__device__ inline bool setup(Lane& L, const Lds& S_lds, const Consts& C, const Inst& I, uint64_t ci, int Ki,
                             double lo, double hi) {
    const int t = lane();
    const int N = I.N, V = I.V, LD = S_lds.LD;
    L.on = t < V;
    const int i = L.on ? t / N : 0, a = L.on ? t % N : 0;
    L.i = i;
    L.a = a;
    const hvp_system& S = I.systems[I.vsys[i]];
    const double ts = S.ts;
    const double v0 = I.x0[2 * i + 1], p0 = I.x0[2 * i];
    L.v0 = v0;
    L.ts = ts;
    L.P1 = p0 + ts * v0;
    L.pmin = S.pmin;
    L.pmax = S.pmax;
    // relaxed steps a, a + 1 of the lane: virtual regions and the interval of v_{a+1}
    int virt0 = -1, virt1 = -1;
    double bm0 = 1.0, bm1 = 1.0, rlo = S.vmin, rhi = S.vmax;
    if (L.on && a + 1 >= Ki) {
        const int kend = a + 1 < N ? a + 1 : N - 1;
        for (int k = Ki; k <= kend; ++k) {
            double nlo, nhi, bm;
            bool dead;
            const int vr = relax_step(S, C, k, lo, hi, nlo, nhi, bm, dead);
            if (dead) break;
            if (k == a) {
                virt0 = vr;
                bm0 = bm;
                rlo = nlo;
                rhi = nhi;
            } else {
                virt1 = vr;
                bm1 = bm;
            }
            lo = nlo;
            hi = nhi;
        }
    }
    auto dyn = [&](int k, double& aa, double& bb, double& cc) {
        const int vr = k == a ? virt0 : virt1;  // k is a or a + 1
        const bool fx = k < Ki;
        const int r = fx ? code_region(ci, k) : (vr >= 0 ? vr : 0);
        const bool on = fx || vr >= 0;
        aa = on ? S.a[r] : 1.0;
        bb = fx ? S.b[r] : (vr >= 0 ? (k == a ? bm0 : bm1) : 1.0);
        cc = on ? S.c[r] : 0.0;
    };
    {
        double aa, bb, cc;
        dyn(a, aa, bb, cc);
        const bool on = a < Ki || virt0 >= 0;
        L.am = aa;
        L.ub = bb;
        L.uc = cc;
        L.ucost = on;
        L.ulo = on ? cc + bb * S.umin : -1e30;
        L.uhi = on ? cc + bb * S.umax : 1e30;
        if (a + 1 < Ki) {
            const int r1 = code_region(ci, a + 1);
            L.vlo = fmax(S.vmin, S.vlo[r1]);
            L.vhi = fmin(S.vmax, S.vhi[r1]);
        } else if (a >= Ki) {  // relaxed v_{a+1}: its reachable interval (v_{Ki}'s is implied)
            L.vlo = fmax(S.vmin, rlo);
            L.vhi = fmin(S.vmax, rhi);
        } else {
            L.vlo = S.vmin;
            L.vhi = S.vmax;
        }
        L.dec = C.dec[a];
        L.acc = C.acc[a];
    }
    // soft safe-distance row of state k = a + 1 (a >= 1: the state depends on y)
    const double P1m = __shfl(L.P1, t >= N ? t - N : t, W);  // P1 of vehicle i-1
    const double P1p = __shfl(L.P1, t + N < W ? t + N : t, W);
    L.sf = 0;
    L.sfd = 0.0;
    if (L.on && a >= 1) {
        if (i >= 1) {
            L.sf = 1;
            L.sfd = -C.d_safe - (L.P1 - P1m);
        } else if (I.lsp && I.L == 0) {
            L.sf = 2;
            L.sfd = I.xl[a + 1] - C.d_safe - L.P1;
        }
    }
    // ---- Hessian row t: closed-form block tridiagonal part
    const Forms F = forms(C, I, i);
    double* Hrow = S_lds.J + (L.on ? t : 0) * LD;
    if (L.on) {
        for (int c = 0; c < V; ++c) {
            const int j = c / N, b = c % N;
            const int mx = a > b ? a : b;
            const double cnt = (double)(N - mx - 1);
            double h = 0.0;
            if (j == i) {
                h = 2.0 * F.Wpp * ts * ts * cnt + (a != b ? 2.0 * ts * F.Wpv : 2.0 * F.Wvv);
            } else if (j == i - 1) {
                h = 2.0 * ts * ts * F.Cpp * cnt + (a < b ? 2.0 * ts * F.Cpv : 0.0) + (b < a ? 2.0 * ts * F.Cvp : 0.0) +
                    (a == b ? 2.0 * F.Cvv : 0.0);
            } else if (j == i + 1) {
                h = 2.0 * ts * ts * F.Cpp * cnt + (b < a ? 2.0 * ts * F.Cpv : 0.0) + (a < b ? 2.0 * ts * F.Cvp : 0.0) +
                    (a == b ? 2.0 * F.Cvv : 0.0);
            }
            Hrow[c] = h;
        }
    }
    // ---- linear term: f = g^v_{a+1} + ts sum_{k >= a+2} g^p_k at y = 0 (p_k = P1, v_k = 0)
    double f = 0.0;
    if (L.on) {
        const double cp = F.Cpp * ((i >= 1 ? P1m : 0.0) + (i + 1 < I.n ? P1p : 0.0));
        const double cv = (i >= 1 ? F.Cvp * P1m : 0.0) + (i + 1 < I.n ? F.Cpv * P1p : 0.0);
        double lp, lv;
        lin(C, I, i, a + 1, lp, lv);
        f = 2.0 * (F.Wpv * L.P1 + lv) + 2.0 * cv;
        for (int k = a + 2; k <= N; ++k) {
            lin(C, I, i, k, lp, lv);
            f += ts * (2.0 * (F.Wpp * L.P1 + lp) + 2.0 * cp);
        }
    }
    // ---- input cost Q_u u^2 (a < K_i) and variation Q_du (du)^2 within the vehicle (hvp_coop.h)
    auto ucoef = [&](int k, double& ub, double& gk, double& gkm) {
        double aa, bb, cc;
        dyn(k, aa, bb, cc);
        const double ib = 1.0 / bb;
        ub = k == 0 ? -(aa * v0 + cc) * ib : -cc * ib;
        gk = ib;
        gkm = k == 0 ? 0.0 : -aa * ib;
    };
    const double w2 = 2.0 * C.Qu;
    const int base = i * N;
    if (L.on) {
        double ub, gk, gkm;
        ucoef(a, ub, gk, gkm);
        if (L.ucost) {
            Hrow[t] += w2 * gk * gk;
            f += w2 * ub * gk;
            if (a >= 1) Hrow[t - 1] += w2 * gk * gkm;
        }
        if (a + 1 < N && (a + 1 < Ki || virt1 >= 0)) {
            double ub1, gk1, gkm1;
            ucoef(a + 1, ub1, gk1, gkm1);
            Hrow[t] += w2 * gkm1 * gkm1;
            f += w2 * ub1 * gkm1;
            Hrow[t + 1] += w2 * gk1 * gkm1;
        }
        if (C.Qdu != 0.0) {
            const double wd = 2.0 * C.Qdu;
            for (int k = a - 1; k <= a + 1; ++k) {
                if (k < 0 || k + 1 >= N || !(k + 1 < Ki)) continue;
                double ubk, gkk, gkmk, ubk1, gkk1, gkmk1;
                ucoef(k, ubk, gkk, gkmk);
                ucoef(k + 1, ubk1, gkk1, gkmk1);
                const double g_kp = gkk1, g_k = gkmk1 - gkk, g_km = k >= 1 ? -gkmk : 0.0;
                const double eb = ubk1 - ubk;
                const double gt = a == k + 1 ? g_kp : (a == k ? g_k : (a == k - 1 ? g_km : 0.0));
                if (gt == 0.0) continue;
                f += wd * eb * gt;
                Hrow[k + 1 - a + t] += wd * gt * g_kp;
                Hrow[k - a + t] += wd * gt * g_k;
                if (k >= 1) Hrow[k - 1 - a + t] += wd * gt * g_km;
            }
        }
    }
    (void)base;
    L.f = L.on ? f : 0.0;
    L.y = 0.0;
    const int bad = L.on && a == 0 && !(L.P1 >= S.pmin - 1e-9 * (1.0 + fabs(S.pmin)) &&
                                         L.P1 <= S.pmax + 1e-9 * (1.0 + fabs(S.pmax)));
    return wor(bad) == 0;
}

// Slacks of lane t's rows and its most violated one (largest violation^2 / |c|^2).
__device__ inline void most_violated(const Lane& L, const Consts& C, double y, double yprev, double p, double pm,
                                     unsigned act, unsigned sat, double tol, double& score, int& id, double& slack) {
    const int t = lane();
    score = -1.0;
    id = -1;
    slack = 0.0;
    if (!L.on) return;
    double best_v2 = 0.0, best_nn = 1.0;
    auto consider = [&](int r, int rid, double s, double nn, double scale) {
        if (((act >> r) & 1u) || !(s < -tol * scale)) return;
        const double v2 = s * s;
        if (id < 0 || v2 * best_nn > best_v2 * nn) {
            id = rid;
            best_v2 = v2;
            best_nn = nn;
            slack = s;
        }
    };
    const int a = L.a;
    const double am = L.am;
    const double gv = y, gu = y - am * yprev, ga = y - yprev;
    const double nu = a ? 1.0 + am * am : 1.0, na = a ? 2.0 : 1.0;
    const int b0 = ROWS * t;
    consider(0, b0 + 0, gv - L.vlo, 1.0, 1.0 + fabs(L.vlo));
    consider(1, b0 + 1, L.vhi - gv, 1.0, 1.0 + fabs(L.vhi));
    consider(2, b0 + 2, gu - L.ulo, nu, 1.0 + fabs(L.ulo) + fabs(am * yprev));
    consider(3, b0 + 3, L.uhi - gu, nu, 1.0 + fabs(L.uhi) + fabs(am * yprev));
    consider(4, b0 + 4, ga - L.dec, na, 1.0 + fabs(yprev));
    consider(5, b0 + 5, L.acc - ga, na, 1.0 + fabs(yprev));
    if (a >= 1) {
        const double nn = L.ts * L.ts * a;
        const double sc = 1.0 + fabs(p);
        consider(6, b0 + 6, p - L.pmin, nn, sc);
        consider(7, b0 + 7, L.pmax - p, nn, sc);
        if (L.sf) {
            // slack d - c.y of the soft row (the constants are folded into sfd)
            const double gap = L.sf == 1 ? (-C.d_safe) - (p - pm) : L.sfd + L.P1 - p;
            const bool sw = sat & 1u;
            consider(8, sw ? (b0 + 8) | REV : b0 + 8, sw ? -gap : gap, L.sf == 1 ? 2.0 * nn : nn, sc);
        }
    }
    if (id >= 0) score = best_v2 / best_nn;
}

// Cooperative Goldfarb-Idnani over the wave (the algorithm of hvp_coop.h::solve).
//
// Early stop (cut < inf): every iterate of the dual method is the optimum of a relaxation of the
// QP (the active rows as inequalities, the saturated soft rows' penalties linear, every other
// soft row's penalty dropped; multipliers feasible), so its objective (direct_cost in dual mode)
// is a lower bound of the QP's optimum.  Every fourth scan the objective is evaluated; once it
// exceeds `cut` the solve returns GI_CUT with that bound in `bound` -- the branch and bound prunes
// such a QP anyway, so the search tree is unchanged.
constexpr int GI_CUT = 9;
__device__ inline double direct_cost(const Lane& L, const Consts& C, const Inst& I, uint64_t ci, int Ki,
                                     double* u_lane, int dual_sat);
__device__ inline int solve(Lane& L, const Lds& Sg, const Consts& C, const Inst& I, int max_iter, int& iters,
                            Prof& pf, int Ki = 0, double cut = __builtin_inf(), double* bound = nullptr) {
    const int t = lane();
    const int N = I.N, V = I.V, LD = Sg.LD;
    iters = 0;
    double* J = Sg.J;
    double* R = Sg.R;
    wsync();
    // ---- Cholesky H = L L' into R (lower, row-major)
    for (int j = 0; j < V; ++j) {
        if (t == j) {
            double s = J[j * LD + j];
            for (int k = 0; k < j; ++k) s -= R[j * LD + k] * R[j * LD + k];
            R[j * LD + j] = s > 0.0 ? sqrt(s) : -1.0;
        }
        wsync();
        const double d = R[j * LD + j];
        if (!(d > 0.0)) return GI_FAIL_CHOL;
        const double dinv = 1.0 / d;
        if (t > j && t < V) {
            double v = J[t * LD + j];
            for (int k = 0; k < j; ++k) v -= R[t * LD + k] * R[j * LD + k];
            R[t * LD + j] = v * dinv;
        }
        wsync();
    }
    pf.mark(1);
    // ---- unconstrained minimiser (lane t holds 1 / L_tt: the substitution chains are a multiply
    // and a readlane per step)
    const double ldinv = t < V ? 1.0 / R[t * LD + t] : 0.0;
    {
        double acc = -L.f, w = 0.0;
        for (int i = 0; i < V; ++i) {
            const double wi = bcu(acc * ldinv, i);
            if (t == i) w = wi;
            if (t > i && t < V) acc -= R[t * LD + i] * wi;
        }
        double acc2 = w;
        L.y = 0.0;
        for (int i = V - 1; i >= 0; --i) {
            const double yi = bcu(acc2 * ldinv, i);
            if (t == i) L.y = yi;
            if (t < i) acc2 -= R[i * LD + t] * yi;
        }
    }
    // ---- J = L^-T (row t of J = column t of L^-1)
    wsync();
    if (t < V) {
        for (int i = 0; i < V; ++i) {
            double v = i == t ? 1.0 : 0.0;
            for (int k = 0; k < i; ++k) v -= R[i * LD + k] * J[t * LD + k];
            J[t * LD + i] = v * bcu(ldinv, i);
        }
    }
    wsync();
    if (t < V)
        for (int c = 0; c < V; ++c) R[t * LD + c] = 0.0;
    wsync();
    double u = 0.0;
    double rinv = 0.0;  // 1 / R[t][t] of active position t (the back substitution's divisions)
    int id = -1;
    int nact = 0;
    unsigned act = 0, sat = 0;
    const double wgt = C.w;
    const double tol = 1e-11;
    int iter = 0, scans = 0;
    for (;;) {
        if (cut < 1e300 && (++scans & 3) == 0) {
            const double lb = direct_cost(L, C, I, 0, Ki, nullptr, (int)(sat & 1u));
            if (lb > cut) {
                iters = iter;
                *bound = lb;
                return GI_CUT;
            }
        }
        pf.mark(2);
        // ---------------- most violated row
        const double yv = t < V ? L.y : 0.0;
        double yprev = shift_up1(yv);
        if (L.a == 0) yprev = L.v0;
        const double cum = vehicle_prefix(yv, N);
        const double p = L.P1 + L.ts * cum;  // p_{i,a+1}
        const double pm = __shfl(p, t >= N ? t - N : t, W);
        double score, bsl;
        int bid;
        most_violated(L, C, yv, yprev, p, pm, act, sat, tol, score, bid, bsl);
        double key = -score;
        int who = t;
        wargmin(key, who);
        if (!(key < 0.0)) break;
        const int pr = bcu(bid, who);
        const int base = pr & (REV - 1);
        const bool rev = (pr & REV) != 0;
        const int owner = base / ROWS, rr = base % ROWS;
        const bool psoft = rr == 8;
        // row normal as up to two segments of lanes: c = cf1 on [s1, s1 + n1), cf2 on [s2, s2 + n2)
        int s1 = owner, n1 = 1, s2 = owner - 1, n2 = 0;
        double cf1 = 0.0, cf2 = 0.0, dloc = 0.0;
        {
            const int oa = owner % N;
            const double flip = rev ? -1.0 : 1.0;
            if (rr < 6) {
                const int pair = rr / 2;
                const double sgn = (rr & 1) ? 1.0 : -1.0;
                const double ra = bcu(pair == 1 ? L.am : (pair == 2 ? 1.0 : 0.0), owner);
                cf1 = flip * sgn;
                n2 = oa >= 1 && pair != 0 ? 1 : 0;
                cf2 = -flip * sgn * ra;
                if (t == owner) {
                    // value selects: opaque copies keep the compiler from turning this into a
                    // select of field addresses (which would put the whole Lane in scratch)
                    double vlo = L.vlo, vhi = L.vhi, ulo = L.ulo, uhi = L.uhi, dlo = L.dec, dhi = L.acc;
                    asm volatile("" : "+v"(vlo), "+v"(vhi), "+v"(ulo), "+v"(uhi), "+v"(dlo), "+v"(dhi));
                    const double lo = pair == 0 ? vlo : (pair == 1 ? ulo : dlo);
                    const double hi = pair == 0 ? vhi : (pair == 1 ? uhi : dhi);
                    const double cst = oa == 0 ? -ra * L.v0 : 0.0;
                    dloc = (rr & 1) ? hi - cst : -(lo - cst);
                }
            } else if (rr < 8) {
                const double sgn = rr == 7 ? 1.0 : -1.0;
                s1 = owner - oa;
                n1 = oa;
                cf1 = flip * sgn * L.ts;
                n2 = 0;
                if (t == owner) dloc = rr == 6 ? L.P1 - L.pmin : L.pmax - L.P1;
            } else {
                s1 = owner - oa;
                n1 = oa;
                cf1 = flip * L.ts;
                const int ksf = bcu(L.sf, owner);
                if (ksf == 1) {
                    s2 = owner - oa - N;
                    n2 = oa;
                    cf2 = -flip * L.ts;
                } else {
                    n2 = 0;
                }
                if (t == owner) dloc = L.sfd;
            }
            dloc = bcu(dloc, owner);
            if (rev) dloc = -dloc;
        }
        auto coef = [&](int j) -> double {
            return (j >= s1 && j < s1 + n1 ? cf1 : 0.0) + (j >= s2 && j < s2 + n2 ? cf2 : 0.0);
        };
        const double np_t = t < V ? -coef(t) : 0.0;
        const double dp = dloc;
        double unew = 0.0;
        for (;;) {
            if (++iter > max_iter) { iters = iter; return GI_FAIL_ITER; }
            pf.mark(3);
            // ---- dv_c = sum_i J[i][c] np_i over the row's support
            double dv = 0.0;
            if (t < V) {
                for (int j = s1; j < s1 + n1; ++j) dv -= J[j * LD + t] * cf1;
                for (int j = s2; j < s2 + n2; ++j) dv -= J[j * LD + t] * cf2;
            }
            Sg.v[t] = dv;
            wsync();
            const double dn = wsum(dv * dv);
            const double d2n = wsum(t >= nact ? dv * dv : 0.0);
            double z = 0.0;
            if (t < V)
                for (int c = nact; c < V; ++c) z += J[t * LD + c] * Sg.v[c];
            pf.mark(4);
            double r = 0.0;
            {
                double accr = t < nact ? dv : 0.0;
                for (int j = nact - 1; j >= 0; --j) {
                    const double rj_ = bcu(accr * rinv, j);
                    if (t == j) r = rj_;
                    if (t < j) accr -= R[t * LD + j] * rj_;
                }
            }
            double k1key = 1e300;
            int k1 = t;
            pf.mark(5);
            // blocking multipliers: r_j above the rounding level of r (a noise-level r_j > 0 with a
            // rounding-level u_j < 0 would give a huge NEGATIVE step), u clamped at 0
            const double rmax = wmax(t < nact ? fabs(r) : 0.0);
            if (t < nact && r > 1e-13 * rmax) k1key = fmax(u, 0.0) / r;
            wargmin(k1key, k1);
            const double t1 = k1key;
            double k3key = 1e300;
            int k3 = t;
            if (t < nact && id >= 0 && (id & (REV - 1)) % ROWS == 8 && r < -1e-13 * rmax)
                k3key = fmax(wgt - u, 0.0) / (-r);
            wargmin(k3key, k3);
            double t3 = k3key;
            bool new_sat = false;
            if (psoft && wgt - unew <= t3) {
                t3 = wgt - unew;
                new_sat = true;
            }
            const bool zstep = d2n > 1e-12 * dn;  // relative: V = 64 rows of rounding in d2n
            const double zn = d2n;
            const double sp_now = dp + wsum(np_t * (t < V ? L.y : 0.0));
            const double t2 = zstep && zn > 0.0 ? fmax(-sp_now, 0.0) / zn : 1e300;
            const double tstep = fmin(t1, fmin(t2, t3));
            if (!(tstep < 1e299)) {
                if (I.debug && I.debug < 3 && t == 0)
                    printf("[cent] GI_FAIL_DUAL iter %d nact %d row %d (owner %d rr %d rev %d) d2n %.3e dn %.3e "
                           "sp %.6e\n", iter, nact, pr, owner, rr, (int)rev, d2n, dn, sp_now);
                if (I.debug == 1 && t < nact) printf("[cent]   act %d: id %d u %.6e r %.6e dv %.6e\n", t, id, u, r, dv);
                if (I.debug == 1 && t < V) printf("[cent]   y %d = %.6e np %.3e\n", t, L.y, np_t);
                iters = iter;
                return GI_FAIL_DUAL;
            }
            if (I.debug == 2 && t == 0)
                printf("[cent] it %d row %d nact %d t1 %.4e(k%d) t2 %.4e t3 %.4e d2n/dn %.3e sp %.4e\n", iter, pr, nact,
                       t1, k1, t2, t3, dn > 0 ? d2n / dn : 0.0, sp_now);
            if (t2 < 1e299 && t < V) L.y += tstep * z;
            if (t < nact) u -= tstep * r;
            unew += tstep;
            if (t2 <= t1 && t2 <= t3) {
                pf.mark(6);
                pf.count(11);
                // ---- add p: one Householder reflection H of J's trailing columns maps
                // d2 = dv[nact..V) onto alpha e_nact (J <- J diag(I, H), R gets the column
                // (dv[0..nact), alpha)).  Every lane updates its own row of J: no serial
                // rotation chain (the lane solver's Givens sweep is V - nact dependent steps).
                const double x0 = Sg.v[nact];
                double alpha = x0;
                if (V - 1 > nact) {
                    alpha = x0 >= 0.0 ? -sqrt(d2n) : sqrt(d2n);
                    const double beta = 1.0 / (d2n - x0 * alpha);  // 2 / v'v, v = d2 - alpha e_0
                    if (t < V) {
                        double w = J[t * LD + nact] * (x0 - alpha);
                        for (int c = nact + 1; c < V; ++c) w += J[t * LD + c] * Sg.v[c];
                        const double bw = beta * w;
                        J[t * LD + nact] -= bw * (x0 - alpha);
                        for (int c = nact + 1; c < V; ++c) J[t * LD + c] -= bw * Sg.v[c];
                    }
                }
                if (t < nact) R[t * LD + nact] = dv;
                if (t == nact) {
                    R[t * LD + nact] = alpha;
                    rinv = 1.0 / alpha;
                }
                if (t == nact) { u = unew; id = pr; }
                if (t == owner) act |= 1u << rr;
                ++nact;
                wsync();
                pf.mark(7);
                break;
            }
            pf.mark(6);
            pf.count(11);
            int drop;
            const bool by_sat = t3 <= t1;
            if (by_sat) {
                if (new_sat) {
                    if (t == owner) sat ^= 1u;
                    wsync();
                    pf.mark(8);
                    break;
                }
                drop = k3;
            } else {
                drop = k1;
            }
            const int dropped = bcu(id, drop);
            {
                const int ob = (dropped & (REV - 1)) / ROWS, brr = (dropped & (REV - 1)) % ROWS;
                if (t == ob) {
                    act &= ~(1u << brr);
                    if (by_sat) sat ^= 1u;
                }
            }
            const double u_n = __shfl_down(u, 1, W);
            const int id_n = __shfl_down(id, 1, W);
            if (t >= drop && t < nact - 1) { u = u_n; id = id_n; }
            if (t == nact - 1) { u = 0.0; id = -1; }
            if (t < V) {
                for (int j = drop; j < nact - 1; ++j) R[t * LD + j] = R[t * LD + j + 1];
                R[t * LD + nact - 1] = 0.0;
            }
            wsync();
            for (int i = drop; i < nact - 1; ++i) {
                double gc, gs;
                givens(R[i * LD + i], R[(i + 1) * LD + i], gc, gs);
                wsync();
                if (t >= i && t < nact - 1) {
                    const double a0 = R[i * LD + t], a1 = R[(i + 1) * LD + t];
                    R[i * LD + t] = gc * a0 + gs * a1;
                    R[(i + 1) * LD + t] = -gs * a0 + gc * a1;
                }
                if (t < V) {
                    const double a0 = J[t * LD + i], a1 = J[t * LD + i + 1];
                    J[t * LD + i] = gc * a0 + gs * a1;
                    J[t * LD + i + 1] = -gs * a0 + gc * a1;
                }
                wsync();
            }
            if (t >= drop && t < nact - 1) rinv = 1.0 / R[t * LD + t];
            --nact;
            pf.mark(8);
        }
    }
    iters = iter;
    int bad = 0;
    if (t < nact) {
        if (u < -1e-9 * wgt) bad = 1;
        if ((id & (REV - 1)) % ROWS == 8 && u > wgt * (1.0 + 1e-9)) bad = 1;
    }
    return wor(bad) ? GI_FAIL_VERIFY : GI_OK;
}

// Objective of the platoon trajectory, term by term (cent_mld.py:83-140; relaxed steps a >= K_i
// carry no input cost).  Lane t adds the terms of state a + 1 of vehicle i and of input a; lane
// a = 0 also those of state 0.  u_lane (optional) receives the lane's input u_{i,a}.
//
// dual_sat >= 0: the objective of a Goldfarb-Idnani iterate instead (solve's early stop): the soft
// safe-distance rows of states >= 2 contribute w (c.y - d) when saturated (bit 0 of dual_sat, the
// lane's own row) and nothing otherwise; the constant rows of states 0 and 1 keep their penalty.
__device__ inline double direct_cost(const Lane& L, const Consts& C, const Inst& I, uint64_t ci, int Ki,
                                     double* u_lane = nullptr, int dual_sat = -1) {
    const int t = lane();
    const int N = I.N;
    const double yv = L.on ? L.y : 0.0;
    double vp = shift_up1(yv);
    if (L.a == 0) vp = L.v0;
    const double cum = vehicle_prefix(yv, N);
    const double pn = L.P1 + L.ts * cum, vn = yv;        // state a + 1
    const double pnm = __shfl(pn, t >= N ? t - N : t, W);  // vehicle i-1, same step
    const double vnm = __shfl(vn, t >= N ? t - N : t, W);
    const double p0 = L.on ? I.x0[2 * L.i] : 0.0, v0 = L.v0;
    const double p0m = L.on && L.i >= 1 ? I.x0[2 * (L.i - 1)] : 0.0, v0m = L.on && L.i >= 1 ? I.x0[2 * L.i - 1] : 0.0;
    const double Qpv2 = 2.0 * C.Qpv;
    auto quad = [&](double ep, double ev) { return C.Qpp * ep * ep + Qpv2 * ep * ev + C.Qvv * ev * ev; };
    // penalty w max(0, g) of a safe row; in dual mode the row of a state >= 2 is the QP's soft row
    auto pen = [&](int k, double g) {
        if (dual_sat < 0 || k < 2) return C.w * fmax(0.0, g);
        return (dual_sat & 1) ? C.w * g : 0.0;
    };
    auto state_terms = [&](int k, double p, double v, double pm, double vm) {
        double Jt = 0.0;
        if (L.i == I.L)
            Jt += quad(p - I.xl[k] + (I.lsp ? C.t0 * v + C.d0 : 0.0), v - I.xl[N + 1 + k]);
        if (L.i >= 1) {
            Jt += quad(p + C.t0 * v + C.d0 - pm, v - vm);
            Jt += pen(k, p - pm + C.d_safe);
        } else if (I.lsp && I.L == 0) {
            Jt += pen(k, p - I.xl[k] + C.d_safe);
        }
        return Jt;
    };
    double Jt = 0.0, u = 0.0;
    if (L.on) {
        Jt += state_terms(L.a + 1, pn, vn, pnm, vnm);
        u = (vn - L.am * vp - L.uc) / L.ub;
        if (L.ucost) Jt += C.Qu * u * u;
        if (L.a == 0) Jt += state_terms(0, p0, v0, p0m, v0m);
    }
    const double uprev = shift_up1(u);
    if (L.on && L.a >= 1 && L.a < Ki) Jt += C.Qdu * (u - uprev) * (u - uprev);
    if (u_lane) *u_lane = u;
    return wsum(Jt);
}

}  // namespace cent
}  // namespace hvp
