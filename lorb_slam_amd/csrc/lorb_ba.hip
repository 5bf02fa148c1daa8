// lorb_ba.hip -- reprojection-error bundle adjustment on gfx950 (MI355X), FP64.
//
// Restates BA::ProjectPoseOptimization (src/bundle_adjust.cpp:158-202) and
// BA::LocalPoseOptimization (src/bundle_adjust.cpp:207-330): ceres::Solve with the default
// trust-region Levenberg-Marquardt options + DENSE_SCHUR.
//
// MI355X-first structure (device-resident LM, batched over independent windows):
//   * every LM scalar decision (accept/reject, radius, tolerances) is made ON THE DEVICE by a
//     one-workgroup-per-window kernel, so an LM iteration is a fixed sequence of launches with
//     no host round trip; it is captured once into a hipGraph and replayed.
//   * point-major Schur: one workgroup per point group linearises its observations, eliminates its
//     points and forms its camera-block partials on chip (k_ba_ls; a group spans <= 128 cameras);
//     one workgroup per band block sums the groups' partials in group order (k_ba_red); the
//     back-substitution re-evaluates the linearisation (k_ba_bs2).  Nothing is stored per
//     observation.  (Round 4's pair-major path -- per-observation tiles, one workgroup per camera
//     block pair over a CSR pair list -- was removed in round 6.)
//   * the reduced camera system is banded (cameras in reverse Cuthill-McKee order): a two-sided
//     band Cholesky with the LM head inside (k_ba_chol_2s), or the wider variants.
//   * all reductions are fixed-order trees (block partials reduced in index order): deterministic,
//     no FP64 atomics.
//
// FP64 contraction: the BA arithmetic may fuse multiply-adds (v_fma_f64; its parity bar is 1e-5
// relative, not bit-exactness -- VERDICT r04 item 3).  The Makefile's global -ffp-contract=off stays
// for the float paths that must be bit-exact (projection, grid, unprojection, ORB, stereo: the other
// translation units).  Everything in this file is deterministic either way (fixed reduction orders);
// the host restatement that must round like the reference (lorb_pose_to_Tcw, cv::Rodrigues) turns
// contraction off in its own body.
#ifndef LORB_NO_CONTRACT  // A/B builds only (tools/isa_fma.py, tools/build_variant.sh nofma -DLORB_NO_CONTRACT)
#pragma clang fp contract(fast)
#endif
#include "lorb_ba_math.h"
#include "lorb_internal.h"


#include <algorithm>
#include <chrono>
#include <cmath>
#include <map>
#include <type_traits>

namespace {

using lorb::residual;
using lorb::residual_jac;
using lorb::residual_jac_s;
using lorb::residual_s;

#ifndef LORB_KGB
#define LORB_KGB 256
#endif
constexpr int kGB = LORB_KGB;  // observations per point group (one workgroup), see K1

struct BaWin {
  int pose_base, n_poses, point_base, n_points;
  int pblk_base, n_pblk;
  int env_base, env_size, n, row_base, bw;  // S band: row i holds cols [i-bw, i]
  int obs_base, n_obs;
  int n_obs_all;  // observations of the window over all ranks (== n_obs unless sharded)
  // point-major path: the window's group partials start at part_base, part_stride doubles per group
  // (camera terms at part_cam within it); bwc = the camera-level half band
  int part_stride, part_cam, bwc, pad_;
  // partial runs ("super-groups"): F consecutive point groups of the window processed by one
  // k_ba_ls workgroup into ONE partial (F = 1: one per group); super-groups [sg_base, sg_base + n_sg)
  int sg_base, n_sg;
  long long part_base;
  double fx, fy, cx, cy;
};
struct PBlk { int win, p0, cnt, o0, no; };  // point group: points [p0, p0+cnt), obs [o0, o0+no)
struct BlockPair { int win, ch, cl, off, cnt; };  // global camera indices, pair list range
struct WinState {
  double radius, decrease_factor, cost, x_norm, gmax, initial_cost;
  int iter, n_success, n_invalid, done, relin, cur, last_successful, term, chol_fail, pad;
};
struct LMOpt {
  int max_iter, max_invalid, jacobi;
  double ftol, gtol, ptol, init_radius, max_radius, min_radius, min_rel, min_diag, max_diag;
};

// Wave reductions, butterfly xor 32, 16, 8, 4, 2, 1, with no LDS traffic.  The cross-row steps
// use gfx950's v_permlane32_swap / v_permlane16_swap on two copies of the value: afterwards lane i
// holds {v_i, v_(i^32)} (resp. i^16) across the two copies.  The in-row steps are DPP moves:
// row_ror:8 is xor 8 within a 16-lane row, and once lanes i and i^8 agree row_ror:4 delivers the
// xor-4 partner's value; quad_perm does xor 2 and xor 1.  Every step combines a lane and its
// partner with a commutative op, so all lanes end with the bits of the plain shuffle butterfly.
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  const unsigned long long u = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)(u & 0xffffffffu), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(u >> 32), CTRL, 0xF, 0xF, false);
  return __longlong_as_double(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}
// {v_i, v_partner} for partner i^32 (W32) or i^16
template <bool W32>
__device__ __forceinline__ void xrow_pair(double v, double& a, double& b) {
  const unsigned long long u = __double_as_longlong(v);
  const unsigned lo = (unsigned)(u & 0xffffffffu), hi = (unsigned)(u >> 32);
  const auto l = W32 ? __builtin_amdgcn_permlane32_swap(lo, lo, false, false)
                     : __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  const auto h = W32 ? __builtin_amdgcn_permlane32_swap(hi, hi, false, false)
                     : __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  a = __longlong_as_double(((unsigned long long)h[0] << 32) | l[0]);
  b = __longlong_as_double(((unsigned long long)h[1] << 32) | l[1]);
}
__device__ __forceinline__ double wave_sum(double v) {
  double a, b;
  xrow_pair<true>(v, a, b); v = a + b;
  xrow_pair<false>(v, a, b); v = a + b;
  v += dpp_d<0x128>(v);  // row_ror:8
  v += dpp_d<0x124>(v);  // row_ror:4
  v += dpp_d<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_d<0xB1>(v);   // quad_perm [1,0,3,2]
  return v;
}
__device__ __forceinline__ double wave_max(double v) {
  double a, b;
  xrow_pair<true>(v, a, b); v = fmax(a, b);
  xrow_pair<false>(v, a, b); v = fmax(a, b);
  v = fmax(v, dpp_d<0x128>(v));
  v = fmax(v, dpp_d<0x124>(v));
  v = fmax(v, dpp_d<0x4E>(v));
  v = fmax(v, dpp_d<0xB1>(v));
  return v;
}
// Reduce-scatter of N <= 32 per-lane values (padded to 32): each step halves the values a lane
// keeps -- the half its partner does not keep goes to the partner, which adds it to its own copy --
// so 32 sums cost 31 exchanges instead of 32 full butterflies.  Partners: lane ^ 32, ^ 16
// (permlane swaps of two different registers), ^ 8 (row_ror:8), the mirrored lane of the half row
// (row_half_mirror: the other quad), ^ 2; a last ^ 1 step completes every sum, and sum k ends in
// lanes 2k, 2k + 1, from where v_readlane broadcasts it.  Every lane returns all N sums.
__device__ __forceinline__ double readlane_d(double v, int l);
__device__ __forceinline__ void swap_pair(double x, double y, bool w32, double& r0, double& r1) {
  const unsigned long long ux = __double_as_longlong(x), uy = __double_as_longlong(y);
  const unsigned xl = (unsigned)ux, xh = (unsigned)(ux >> 32), yl = (unsigned)uy, yh = (unsigned)(uy >> 32);
  const auto l = w32 ? __builtin_amdgcn_permlane32_swap(xl, yl, false, false)
                     : __builtin_amdgcn_permlane16_swap(xl, yl, false, false);
  const auto h = w32 ? __builtin_amdgcn_permlane32_swap(xh, yh, false, false)
                     : __builtin_amdgcn_permlane16_swap(xh, yh, false, false);
  r0 = __longlong_as_double(((unsigned long long)h[0] << 32) | l[0]);
  r1 = __longlong_as_double(((unsigned long long)h[1] << 32) | l[1]);
}
template <int CTRL, int BIT, int H>
__device__ __forceinline__ void rs_dpp_step(double (&v)[32], int lane) {
  const bool up = (lane >> BIT) & 1;
#pragma unroll
  for (int k = 0; k < H; ++k) {
    const double keep = up ? v[k + H] : v[k], send = up ? v[k] : v[k + H];
    v[k] = keep + dpp_d<CTRL>(send);
  }
}
// in place: v[0 .. N) in, the N sums out in every lane (v[N .. 32) are scratch)
template <int N>
__device__ __forceinline__ void wave_sum_all(double (&v)[32]) {
  static_assert(N <= 32, "at most 32 values");
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int k = N; k < 32; ++k) v[k] = 0.0;
#pragma unroll
  for (int k = 0; k < 16; ++k) {  // ^32: lanes < 32 keep k, lanes >= 32 keep k + 16
    double a, b;
    swap_pair(v[k], v[k + 16], true, a, b);
    v[k] = a + b;
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {   // ^16 (rows of 16): even rows keep k, odd rows k + 8
    double a, b;
    swap_pair(v[k], v[k + 8], false, a, b);
    v[k] = a + b;
  }
  rs_dpp_step<0x128, 3, 4>(v, lane);  // row_ror:8 = ^8
  rs_dpp_step<0x141, 2, 2>(v, lane);  // row_half_mirror: the other quad of the half row
  rs_dpp_step<0x4E, 1, 1>(v, lane);   // quad_perm [2,3,0,1] = ^2
  v[0] += dpp_d<0xB1>(v[0]);          // quad_perm [1,0,3,2] = ^1
  // lane l now holds sum (16 b5 + 8 b4 + 4 b3 + 2 b2 + b1) = l >> 1
  const double r = v[0];
#pragma unroll
  for (int k = 0; k < N; ++k) v[k] = readlane_d(r, 2 * k);
}
template <int N>
__device__ __forceinline__ void block_sum(double (&v)[N], double* sh /* [N*256] */) {
  // deterministic fixed tree over a 256-thread block
  const int t = threadIdx.x;
#pragma unroll
  for (int k = 0; k < N; ++k) sh[k * 256 + t] = v[k];
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (t < s) {
#pragma unroll
      for (int k = 0; k < N; ++k) sh[k * 256 + t] += sh[k * 256 + t + s];
    }
    __syncthreads();
  }
#pragma unroll
  for (int k = 0; k < N; ++k) v[k] = sh[k * 256];
  __syncthreads();
}

// sym 3x3 packed (xx,xy,xz,yy,yz,zz) inverse via Cholesky; returns false if not PD
__device__ __forceinline__ bool inv3(const double a[6], double inv[6]) {
  const double l00 = a[0];
  if (!(l00 > 0.0)) return false;
  const double L00 = sqrt(l00);
  const double L10 = a[1] / L00, L20 = a[2] / L00;
  const double d1 = a[3] - L10 * L10;
  if (!(d1 > 0.0)) return false;
  const double L11 = sqrt(d1);
  const double L21 = (a[4] - L20 * L10) / L11;
  const double d2 = a[5] - L20 * L20 - L21 * L21;
  if (!(d2 > 0.0)) return false;
  const double L22 = sqrt(d2);
  // inverse of L (lower)
  const double i00 = 1.0 / L00, i11 = 1.0 / L11, i22 = 1.0 / L22;
  const double i10 = -L10 * i00 * i11;
  const double i21 = -L21 * i11 * i22;
  const double i20 = -(L20 * i00 + L21 * i10) * i22;
  // A^-1 = Li^T Li
  inv[0] = i00 * i00 + i10 * i10 + i20 * i20;
  inv[1] = i10 * i11 + i20 * i21;
  inv[2] = i20 * i22;
  inv[3] = i11 * i11 + i21 * i21;
  inv[4] = i21 * i22;
  inv[5] = i22 * i22;
  return true;
}
__device__ __forceinline__ double s3(const double m[6], int a, int b) {
  if (a > b) { const int t = a; a = b; b = t; }
  return m[a * 3 - (a * (a - 1)) / 2 + (b - a)];  // packed (xx,xy,xz,yy,yz,zz)
}

// ------------------------------------------------------------------------------------------
struct BaDev {
  lorb::RotJet* rot_lin;           // Ctot: rotation state (with d/daa) of x_pose[cur], per linearisation
  lorb::RotVal* rot_cand;          // Ctot: rotation state of the candidate pose x_pose[cur ^ 1]
  lorb::RotJet* rot_fix;           // NF: rotation states of the fixed poses (k_ba_init; they never change)
  lorb::RotVal* rotv_fix;          // NF: the same, value only (the candidate cost)
  const BaWin* win;
  const PBlk* pblk;
  const int* obs_pt;         // K  (global point of each observation)
  const BlockPair* bp;
  const int* pt_obs_off;     // Ptot+1
  const int* obs_cam;        // K  (global optimised camera or -1)
  const int* obs_fix;        // K  (global fixed pose or -1)
  const double2* obs_uv;     // K
  const double* fixed_pose;  // NF*6
  double* x_init_pose;       // Ctot*6 (initial values, never written)
  double* x_init_pt;         // Ptot*3
  double* x_pose[2];         // Ctot*6
  double* x_pt[2];           // Ptot*3
  double* scale_pose;        // Ctot*6
  double* scale_pt;          // Ptot*3
  double* etb;               // Ptot*3 (unscaled)
  double* pinv;              // Ptot*6
  double* U;                 // Ctot*21 (unscaled, packed upper row-major)
  double* V;                 // Ctot*6
  double* env;               // S envelopes (all-reduced when sharded)
  double* rhs;               // sum n
  // sharded plans: kernels write the *_part buffers, the all-reduce produces the
  // global ones (unsharded: *_part == global).  Contiguous per exchange:
  //   lin   [U | V | wlin (2W: cost, point |x|^2)]  sum;   wmax (W: point gradient max)  max
  //   solve [env | rhs | wfail (W)]                 sum
  //   step  wstep (3W: model cost change, candidate cost, point |step|^2)  sum
  double *U_part, *V_part, *wlin, *wlin_part, *wmax, *wmax_part;
  double *env_part, *rhs_part, *wfail, *wfail_part, *wstep, *wstep_part;
  const int* cam_active;     // Ctot: camera observed by some rank
  int sharded, rank0;
  double* ycam;              // sum n (solution, scaled space, y = -step)
  double* part;              // n_pblk * 8 partials
  unsigned long long* dbg;   // diagnostic stamps (LORB_CHOL_STAMPS builds only)
  double* kco;               // k_ba_chol_2s back-substitution operators: per window
                             // ((row_base >> 4) + w) * 1024 doubles, top side's blocks then the
                             // bottom side's, [block][16][64] (BandSide::bsk_block)
  WinState* st;
  // partials (k_ba_ls -> k_ba_red), per super-group (its first camera - pose_base, camera span)
  double* gpart;
  int2* gspan;
  const int4* sgrp;          // per super-group: window, first point group, point groups
  lorb_lm_iteration* trace;  // per window LORB_LM_TRACE_CAP records (lm_decide)
  // [0] point groups, [1] block pairs, [2] super-groups in use.  Launch grids may be larger (device-built plans
  // launch at capacity so that the captured LM graph survives a rebuild); the extra workgroups exit.
  const int* live;
};

__device__ __forceinline__ int u21(int a, int b) {  // packed upper index of 6x6 sym
  if (a > b) { const int t = a; a = b; b = t; }
  return a * 6 - (a * (a - 1)) / 2 + (b - a);
}

// K0: start of a solve, one launch: window states, x[0] <- the initial values, and the
// per-camera rotation states of that first linearisation point (transcendentals once per
// camera; later ones come from k_ba_lm_end on acceptance).
__device__ __forceinline__ void init_run(const BaDev& d, int W, int ctot, int n_pt, int nf, const LMOpt& o, const int i,
                                         const int stride) {
  if (i < W) {
    WinState s;
    s.radius = o.init_radius; s.decrease_factor = 2.0; s.cost = 0.0; s.x_norm = 0.0; s.gmax = 0.0;
    s.initial_cost = 0.0; s.iter = 0; s.n_success = 0; s.n_invalid = 0;
    s.done = d.win[i].n_obs_all == 0 ? 1 : 0;
    s.relin = 1; s.cur = 0; s.last_successful = 1; s.term = 0; s.chol_fail = 0; s.pad = 0;
    d.st[i] = s;
    if (d.sharded) d.wfail_part[i] = 0.0;  // point-block failures (set by k_ba_ls, cleared by k_ba_lm_end)
  }
  if (i < ctot) {
    double x[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) { x[k] = d.x_init_pose[6 * i + k]; d.x_pose[0][6 * i + k] = x[k]; }
    d.rot_lin[i] = lorb::rot_jet(x);
  }
  if (i < nf) {  // the fixed poses' rotation states, once per solve (k_ba_ls / k_ba_bs2 read them)
    double x[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) x[k] = d.fixed_pose[6 * i + k];
    d.rot_fix[i] = lorb::rot_jet(x);
    d.rotv_fix[i] = lorb::rot_val(x);
  }
  for (int k = i; k < 3 * n_pt; k += stride) d.x_pt[0][k] = d.x_init_pt[k];
}
__global__ __launch_bounds__(256) void k_ba_init(BaDev d, int W, int ctot, int n_pt, int nf, LMOpt o) {
  init_run(d, W, ctot, n_pt, nf, o, blockIdx.x * blockDim.x + threadIdx.x, gridDim.x * blockDim.x);
}

// Point groups (PBlk): consecutive points of one window whose observations (contiguous, sorted
// by point) number <= kGB, processed by one 256-thread workgroup: observation-parallel phases
// (thread = observation, coalesced, no serial load chains) alternate with point phases (thread =
// point) that reduce their observations from LDS serially in observation order -- the same
// summation order as a point-serial loop.  A point with more than kGB observations gets a group
// of its own and the observation phases loop over chunks.

// deterministic point-group reductions (fixed butterfly per wave, fixed wave order) over the
// kGB / 64 waves of a point-group workgroup
constexpr int kGW = kGB / 64;
static_assert(kGW >= 1 && kGW <= 16 && kGB % 64 == 0, "point groups of 64..1024 observations, whole waves");
// three block reductions behind one LDS exchange (M1: the second is a max): per-wave butterfly,
// then the waves' values in wave order
template <bool M1>
__device__ __forceinline__ void block_red3(double& a, double& b, double& c, double (*red)[kGW]) {
  a = wave_sum(a); b = M1 ? wave_max(b) : wave_sum(b); c = wave_sum(c);
  if (kGW == 1) return;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) {
    const int w = threadIdx.x >> 6;
    red[0][w] = a; red[1][w] = b; red[2][w] = c;
  }
  __syncthreads();
  a = red[0][0]; b = red[1][0]; c = red[2][0];
#pragma unroll
  for (int k = 1; k < kGW; ++k) { a += red[0][k]; b = M1 ? fmax(b, red[1][k]) : b + red[1][k]; c += red[2][k]; }
}

// Point-block prep (k_ba_ls phase B): the point's scaled E^T E + D^2 inverted at the current
// radius.  Returns false when the 3x3 block is not invertible (Ei = 0).
__device__ __forceinline__ bool prep_point(const double (&Eu)[6], const double (&bu)[3], const double (&sp)[3],
                                           double rad, const LMOpt& o, double (&Ei)[6], double (&b)[3]) {
  double E[6];
#pragma unroll
  for (int k = 0; k < 3; ++k) b[k] = bu[k] * sp[k];
  E[0] = Eu[0] * sp[0] * sp[0]; E[1] = Eu[1] * sp[0] * sp[1]; E[2] = Eu[2] * sp[0] * sp[2];
  E[3] = Eu[3] * sp[1] * sp[1]; E[4] = Eu[4] * sp[1] * sp[2]; E[5] = Eu[5] * sp[2] * sp[2];
  E[0] += fmin(fmax(E[0], o.min_diag), o.max_diag) / rad;
  E[3] += fmin(fmax(E[3], o.min_diag), o.max_diag) / rad;
  E[5] += fmin(fmax(E[5], o.min_diag), o.max_diag) / rad;
  if (!inv3(E, Ei)) {
#pragma unroll
    for (int k = 0; k < 6; ++k) Ei[k] = 0.0;
    return false;
  }
  return true;
}
__device__ __forceinline__ void prep_fail(const BaDev& d, int win) {
  // benign race: every writer stores the same value; sharded plans reduce the flag (K5).  The
  // flag is cleared by k_ba_lm_end (and k_ba_init), not by k_ba_lm_begin: k_ba_ls sets it
  // before k_ba_lm_begin runs.
  if (d.sharded) d.wfail_part[win] = 1.0;
  else d.st[win].chol_fail = 1;
}
// Lane-strided partial sums over a window's point groups (b = lane, lane + 64, ... in that order,
// the per-lane order of a plain loop) with the loads of kPU groups issued before any is added: the
// partials come from the previous kernel (another XCD's L2), so a load-add loop pays one memory
// round trip per step.  F0..F2 pick the fields; M1: field 1 is a max.
template <int F0, int F1, int F2, bool M1>
__device__ __forceinline__ void group_partials(const double* __restrict__ part, int base, int n, int lane,
                                               double& a, double& b, double& c) {
  constexpr int kPU = 8;
  for (int b0 = lane; b0 < n; b0 += 64 * kPU) {
    double v0[kPU], v1[kPU], v2[kPU];
#pragma unroll
    for (int u = 0; u < kPU; ++u) {
      const int g = b0 + 64 * u;
      const double* P = part + 8 * (base + (g < n ? g : 0));
      v0[u] = P[F0]; v1[u] = P[F1]; v2[u] = P[F2];
    }
#pragma unroll
    for (int u = 0; u < kPU; ++u)
      if (b0 + 64 * u < n) {
        a += v0[u];
        b = M1 ? fmax(b, v1[u]) : b + v1[u];
        c += v2[u];
      }
  }
}

// K2b (sharded plans): per-window reduction of the point-group partials of one phase into the
// exchange buffers (PH 0: cost, point |x|^2 (sum) and point gradient max; PH 1: model cost
// change, candidate cost, point |step|^2), fixed lane order + butterfly.
template <int PH>
__global__ __launch_bounds__(64) void k_ba_win_reduce(BaDev d) {
  const int w = blockIdx.x;
  if (d.st[w].done) return;
  const BaWin& W = d.win[w];
  const int lane = threadIdx.x;
  double a = 0.0, b = 0.0, c = 0.0;
  if (PH == 0) group_partials<0, 1, 2, true>(d.part, W.pblk_base, W.n_pblk, lane, a, c, b);
  else group_partials<3, 4, 5, false>(d.part, W.pblk_base, W.n_pblk, lane, a, b, c);
  a = wave_sum(a); b = wave_sum(b);
  c = PH == 0 ? wave_max(c) : wave_sum(c);
  if (lane == 0) {
    if (PH == 0) { d.wlin_part[2 * w] = a; d.wlin_part[2 * w + 1] = b; d.wmax_part[w] = c; }
    else { d.wstep_part[3 * w] = a; d.wstep_part[3 * w + 1] = b; d.wstep_part[3 * w + 2] = c; }
  }
}

// K3: per-window iteration head: finalise the (re)linearisation, termination checks
// Camera terms (gradient max, |x|^2, iteration-0 Jacobi scale) come from the (all-reduced)
// U / V blocks; point terms from the point-group partials (SH: from the exchange buffers).
// One wavefront; returns the state after the head (lane 0 has stored it).  k_ba_lm_begin runs it
// as a kernel; the fused iteration runs it on an otherwise idle wave of the Cholesky (lm_head).
template <bool SH>
__device__ __forceinline__ WinState lm_head(const BaDev& d, const LMOpt& o, int w, int lane, WinState S, const BaWin& W) {
  if (S.relin) {
    // fixed lane assignment + fixed butterfly => deterministic
    double cost = 0.0, gm = 0.0, xn2 = 0.0;
    if (!SH) group_partials<0, 1, 2, true>(d.part, W.pblk_base, W.n_pblk, lane, cost, gm, xn2);
    const int cur = S.cur;
    for (int c = W.pose_base + lane; c < W.pose_base + W.n_poses; c += 64) {
      if (S.iter == 0) {
        const int dg[6] = {0, 6, 11, 15, 18, 20};
        for (int k = 0; k < 6; ++k) d.scale_pose[6 * c + k] = 1.0 / (1.0 + sqrt(d.U[21 * c + dg[k]]));
      }
      if (!d.cam_active[c]) continue;
      for (int k = 0; k < 6; ++k) {
        const double x = d.x_pose[cur][6 * c + k];
        gm = fmax(gm, fabs(x - (x + -d.V[6 * c + k])));
        xn2 += x * x;
      }
    }
    cost = wave_sum(cost); gm = wave_max(gm); xn2 = wave_sum(xn2);
    if (SH) { cost += d.wlin[2 * w]; xn2 += d.wlin[2 * w + 1]; gm = fmax(gm, d.wmax[w]); }
    S.cost = cost;
    S.gmax = gm;
    S.x_norm = sqrt(xn2);
    if (S.iter == 0) S.initial_cost = cost;
    S.last_successful = 1;
    S.relin = 0;
  }
  if (lane == 0) {
    if (S.iter >= o.max_iter) { S.done = 1; S.term = LORB_TERM_NO_CONVERGENCE; }
    else if (S.last_successful && S.gmax <= o.gtol) { S.done = 1; S.term = LORB_TERM_GRADIENT_TOL; }
    else if (S.radius <= o.min_radius) { S.done = 1; S.term = LORB_TERM_MIN_RADIUS; }
    else S.iter++;
    d.st[w] = S;
  }
  return S;
}

template <bool SH>
__device__ __forceinline__ void lm_begin_run(const BaDev& d, const LMOpt& o, const int w) {
  const WinState* Sp = d.st + w;
  const WinState S = *Sp;
  const BaWin W = d.win[w];  // issued with the state, before the done test
  if (S.done) return;
  (void)lm_head<SH>(d, o, w, threadIdx.x, S, W);
}
template <bool SH>
__global__ __launch_bounds__(64) void k_ba_lm_begin(BaDev d, LMOpt o) {
  lm_begin_run<SH>(d, o, blockIdx.x);
}

typedef double v4d __attribute__((ext_vector_type(4)));

__device__ __forceinline__ double& band(double* A, int bw, int i, int j) {
  return A[(size_t)i * (bw + 1) + (j - i + bw)];
}

__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
  __builtin_amdgcn_wave_barrier();
}

// v_rsq_f64 is accurate to about 2^-22 relative; each Newton step squares the error.  Two steps
// reach full double precision; LORB_RSQ_STEPS=1 stops at ~1e-14.
#ifndef LORB_RSQ_STEPS
#define LORB_RSQ_STEPS 2
#endif
__device__ __forceinline__ double rsqrt_refined(double a) {
  double y = __builtin_amdgcn_rsq(a);
#pragma unroll
  for (int s = 0; s < LORB_RSQ_STEPS; ++s) {
    const double e = fma(-a * y, y, 1.0);
    y = fma(0.5 * y, e, y);
  }
  return y;
}

// broadcast lane `l` (wave-uniform) of a double through two v_readlane_b32
__device__ __forceinline__ double readlane_d(double v, int l) {
  const unsigned long long u = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(u & 0xffffffffu), l);
  const int hi = __builtin_amdgcn_readlane((int)(u >> 32), l);
  return __longlong_as_double(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}

// K6: banded Cholesky of S + forward/back substitution; one 256-thread workgroup per window.
// Right-looking with panel width NB.  Wave 0 factors the panel entirely in registers (lane l
// owns panel rows kb+l+64r, r < RPL; the pivot column is broadcast with v_readlane), with the
// forward substitution fused in; rsqrt-refined pivots keep IEEE div/sqrt off the critical
// path.  All four waves then apply the rank-NB trailing update from LDS.
constexpr int NB = 16;

// One 16x16 tile (I, J) of the panel's trailing update (SYRK): A(i, j) -= sum_k L(i, k) L(j, k)
// for ke <= j <= i <= rlast, k in [kb, kb + NB), on v_mfma_f64_16x16x4f64 (K = NB = 4 MFMAs).
// Operand lane l holds row (l & 15), k = l >> 4; accumulator register r holds row
// 4r + (l >> 4), column l & 15.  Entries outside the band / triangle are fed as 0 and never
// stored.
__device__ __forceinline__ void chol_trail_tile(double* A, int bw, int kb, int ke, int rlast,
                                                int I, int J, int lane) {
  if (16 * (I - J) - 15 > bw) return;  // tile entirely outside the band
  const int ci = lane & 15, ck = lane >> 4;
  const int i0 = ke + 16 * I, j0 = ke + 16 * J;
  v4d acc;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = i0 + ck + 4 * r, j = j0 + ci;
    const bool ok = i <= rlast && j <= i && i - j <= bw;
    const double v = band(A, bw, ok ? i : ke, ok ? j : ke);
    acc[r] = ok ? v : 0.0;
  }
#pragma unroll
  for (int kk = 0; kk < NB / 4; ++kk) {
    const int k = kb + 4 * kk + ck;
    const int ia = i0 + ci, jb = j0 + ci;
    const bool oka = ia <= rlast && ia - k <= bw, okb = jb <= rlast && jb - k <= bw;
    const double a = band(A, bw, oka ? ia : k, k), b = band(A, bw, okb ? jb : k, k);
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(oka ? -a : 0.0, okb ? b : 0.0, acc, 0, 0, 0);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = i0 + ck + 4 * r, j = j0 + ci;
    if (i <= rlast && j <= i && i - j <= bw) band(A, bw, i, j) = acc[r];
  }
}

template <bool IN_LDS, int RPL>
__global__ __launch_bounds__(256) void k_ba_chol(BaDev d) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  __shared__ int s_fail;
  __shared__ __attribute__((aligned(16))) double s_col[80];
  __shared__ double s_l[NB][NB + 1], s_zk[NB], s_y[NB];  // a factored panel's diagonal block (extra rows)
  const int w = blockIdx.x;
  if (d.st[w].done) return;
  if (d.sharded && d.wfail[w] > 0.0) {  // a rank's point block was not PD: the step is invalid
    if (threadIdx.x == 0) d.st[w].chol_fail = 1;
    return;
  }
  const BaWin W = d.win[w];
  const int n = W.n, bw = W.bw;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  double *A, *z, *invd;
  if (IN_LDS) {
    A = smem;
    z = smem + (size_t)n * (bw + 1);
    invd = z + n;
    const double* src = d.env + W.env_base;
    for (int k = t; k < n * (bw + 1); k += 256) A[k] = src[k];
    for (int k = t; k < n; k += 256) z[k] = d.rhs[W.row_base + k];
  } else {
    A = d.env + W.env_base;
    z = d.rhs + W.row_base;
    invd = d.ycam + W.row_base;  // scratch, overwritten with the solution at the end
  }
  if (t == 0) s_fail = 0;
  __syncthreads();
#ifdef LORB_CHOL_STAMPS
  const unsigned long long T0 = __builtin_amdgcn_s_memtime();
  unsigned long long tst0 = 0, tst_panel = 0, tst_trail = 0;
#endif
  // Lookahead: panel p's trailing update is split into the tiles covering panel p+1's columns
  // (J = 0, all four waves, before panel p+1) and the rest (J >= 1), which waves 1-3 apply
  // while wave 0 factors panel p+1 -- they touch disjoint columns.
  int pkb = -1, pke = 0, prl = 0;  // previous panel (deferred tiles), pkb < 0: none
  for (int kb = 0; kb < n; kb += NB) {
#ifdef LORB_CHOL_STAMPS
    if (t == 0 && kb == 0) { d.dbg[8 * w] = __builtin_amdgcn_s_memtime() - T0; tst0 = __builtin_amdgcn_s_memtime(); }
#endif
    const int ke = min(kb + NB, n);
    const int rlast = min(n - 1, ke - 1 + bw);
    if (wv != 0 && pkb >= 0) {
      const int m = ((prl - pke + 1 + 15) >> 4) - 1;  // J >= 1 tiles: triangle of side m
      for (int tt = wv - 1; tt < m * (m + 1) / 2; tt += 3) {
        int I = 0;
        while ((I + 1) * (I + 2) / 2 <= tt) ++I;
        chol_trail_tile(A, bw, pkb, pke, prl, I + 1, tt - I * (I + 1) / 2 + 1, lane);
      }
    }
    if (wv == 0) {
      double P[RPL][NB], zr[RPL];
#pragma unroll
      for (int r = 0; r < RPL; ++r) {
        const int row = kb + lane + 64 * r;
        const bool vr = row <= rlast;
#pragma unroll
        for (int q = 0; q < NB; ++q) {
          const int col = kb + q;
          P[r][q] = (vr && col < ke && col <= row && row - col <= bw) ? band(A, bw, row, col) : 0.0;
        }
        zr[r] = vr ? z[row] : 0.0;
      }
      bool bad = false;
      if (ke - kb == NB) {
        // Full panel: one basic block (no per-column branches, pivots via v_readlane), so the
        // compiler can overlap column q+1's pivot chain with column q's bulk updates.  A
        // non-positive pivot turns into NaNs that are never stored: `bad` aborts below.
        // Lanes l < q hold finished or upper-triangle garbage in P[0][q..]; those entries are
        // never read as a pivot/head and never stored, so only z needs masking.
        double yq = 0.0;
#pragma unroll
        for (int q = 0; q < NB; ++q) {
          const double akk = readlane_d(P[0][q], q);
          bad |= !(akk > 0.0);
          const double y = rsqrt_refined(akk);
#pragma unroll
          for (int r = 0; r < RPL; ++r) P[r][q] *= y;  // lane q: akk * y = L(k, k)
          yq = lane == q ? y : yq;
          const double zk = readlane_d(zr[0], q) * y;
          zr[0] = lane > q ? fma(-P[0][q], zk, zr[0]) : (lane == q ? zk : zr[0]);
#pragma unroll
          for (int r = 1; r < RPL; ++r) zr[r] = fma(-P[r][q], zk, zr[r]);
#pragma unroll
          for (int q2 = q + 1; q2 < NB; ++q2) {
            const double l = readlane_d(P[0][q], q2);
#pragma unroll
            for (int r = 0; r < RPL; ++r) P[r][q2] = fma(-P[r][q], l, P[r][q2]);
          }
        }
        if (lane < NB) invd[kb + lane] = yq;
      } else {
#pragma unroll
      for (int q = 0; q < NB; ++q) {
        const int k = kb + q;
        if (k < ke && !bad) {
          const double akk = readlane_d(P[0][q], q);
          if (!(akk > 0.0)) {
            bad = true;
          } else {
            const double y = rsqrt_refined(akk);
#pragma unroll
            for (int r = 0; r < RPL; ++r) {
              const int row = kb + lane + 64 * r;
              if (row > k) P[r][q] *= y;
            }
            if (lane == q) { P[0][q] = akk * y; zr[0] *= y; invd[k] = y; s_col[64] = zr[0]; }
            // broadcast the column head L(kb+q2, k) and z_k through LDS (one write, wide reads)
            s_col[lane] = P[0][q];
            wave_sync_lds();
            const double zk = s_col[64];
            double l[NB];
#pragma unroll
            for (int q2 = q + 1; q2 < NB; ++q2) l[q2] = s_col[q2];
#pragma unroll
            for (int r = 0; r < RPL; ++r) {
              const int row = kb + lane + 64 * r;
              if (row > k) zr[r] -= P[r][q] * zk;
            }
#pragma unroll
            for (int q2 = q + 1; q2 < NB; ++q2) {
#pragma unroll
              for (int r = 0; r < RPL; ++r) {
                const int row = kb + lane + 64 * r;
                if (row >= kb + q2) P[r][q2] -= P[r][q] * l[q2];
              }
            }
            wave_sync_lds();  // all reads of s_col done before the next column overwrites it
          }
        }
      }
      }
#pragma unroll
      for (int r = 0; r < RPL; ++r) {
        const int row = kb + lane + 64 * r;
        if (row <= rlast) {
#pragma unroll
          for (int q = 0; q < NB; ++q) {
            const int col = kb + q;
            if (col < ke && col <= row && row - col <= bw) band(A, bw, row, col) = P[r][q];
          }
          z[row] = zr[r];
        }
      }
      // Rows below the register panel (bw + NB > 64 RPL: a dense window of more than ~80 cameras):
      // the panel's column operations replayed 64 rows at a time from its diagonal block (L(kb+q2,
      // kb+q) in lane q2's P[0][q], z_k in lane q's zr[0], 1 / L(k, k) in invd) -- per row the same
      // operations in the same order as a register row's.
      if (!bad && kb + 64 * RPL <= rlast) {
        const int nq = ke - kb;
        if (lane < NB) {
#pragma unroll
          for (int q = 0; q < NB; ++q) s_l[lane][q] = P[0][q];
          s_zk[lane] = zr[0];
          s_y[lane] = lane < nq ? invd[kb + lane] : 0.0;
        }
        wave_sync_lds();
        for (int r0 = kb + 64 * RPL; r0 <= rlast; r0 += 64) {
          const int row = r0 + lane;
          const bool vr = row <= rlast;
          double X[NB], zx = vr ? z[row] : 0.0;
#pragma unroll
          for (int q = 0; q < NB; ++q) X[q] = (vr && q < nq && row - (kb + q) <= bw) ? band(A, bw, row, kb + q) : 0.0;
#pragma unroll
          for (int q = 0; q < NB; ++q) {
            if (q < nq) {
              X[q] *= s_y[q];
              zx = fma(-X[q], s_zk[q], zx);
#pragma unroll
              for (int q2 = q + 1; q2 < NB; ++q2) X[q2] = fma(-X[q], s_l[q2][q], X[q2]);
            }
          }
          if (vr) {
#pragma unroll
            for (int q = 0; q < NB; ++q)
              if (q < nq && row - (kb + q) <= bw) band(A, bw, row, kb + q) = X[q];
            z[row] = zx;
          }
        }
        wave_sync_lds();
      }
      if (bad && lane == 0) s_fail = 1;
    }
    __syncthreads();
    if (s_fail) break;
#ifdef LORB_CHOL_STAMPS
    if (t == 0) { const unsigned long long q_ = __builtin_amdgcn_s_memtime(); tst_panel += q_ - tst0; tst0 = q_; }
#endif
    // trailing tiles over panel p+1's columns (J = 0); the rest is deferred (see above)
    {
      const int nt = (rlast - ke + 1 + 15) >> 4;
      for (int I = wv; I < nt; I += 4) chol_trail_tile(A, bw, kb, ke, rlast, I, 0, lane);
      pkb = kb; pke = ke; prl = rlast;
    }
    __syncthreads();
#ifdef LORB_CHOL_STAMPS
    if (t == 0) { const unsigned long long q_ = __builtin_amdgcn_s_memtime(); tst_trail += q_ - tst0; tst0 = q_; }
#endif
  }
  if (s_fail) {
    if (t == 0) d.st[w].chol_fail = 1;
    return;
  }
#ifdef LORB_CHOL_STAMPS
  if (t == 0) { d.dbg[8 * w + 2] = tst_trail; d.dbg[8 * w + 1] = tst_panel; }
#endif
  // back substitution L^T y = z, 64-row register blocks from the bottom (wave 0)
  if (wv == 0) {
    for (int bb = ((n - 1) / 64) * 64; bb >= 0; bb -= 64) {
      const int row = bb + lane;
      const int be = min(n - 1, bb + 63);
      double zr = row < n ? z[row] : 0.0;
      // 8-row chunks: the chunk's L(k, row) and 1/L(k, k) are loaded before the serial
      // readlane chain so LDS/global latency is paid once per chunk, not once per row.
      constexpr int BC = 8;
      for (int k0 = be; k0 >= bb; k0 -= BC) {
        double lk[BC], iv[BC];
#pragma unroll
        for (int u = 0; u < BC; ++u) {
          const int k = max(k0 - u, bb);
          const bool ok = k0 - u >= bb && row < k && k - row <= bw;
          lk[u] = band(A, bw, k, ok ? row : k);
          lk[u] = ok ? lk[u] : 0.0;
          iv[u] = invd[k];
        }
#pragma unroll
        for (int u = 0; u < BC; ++u) {
          const int k = k0 - u;
          if (k >= bb) {
            const double yk = readlane_d(zr, k - bb) * iv[u];
            zr = lane == k - bb ? yk : fma(-lk[u], yk, zr);
          }
        }
      }
      if (row < n) z[row] = zr;
      wave_sync_lds();
      // rows above the block: z_i -= sum_k L(k, i) y_k, k in [bb, be], k - i <= bw
      for (int i = max(0, bb - bw) + lane; i < bb; i += 64) {
        double acc = 0.0;
        const int kend = min(be, i + bw);
        for (int k = bb; k <= kend; k += BC) {
          double a[BC], zk[BC];
#pragma unroll
          for (int u = 0; u < BC; ++u) {
            const int kk = min(k + u, kend);
            a[u] = band(A, bw, kk, i);
            zk[u] = z[kk];
          }
#pragma unroll
          for (int u = 0; u < BC; ++u) acc = fma(k + u <= kend ? a[u] : 0.0, zk[u], acc);
        }
        z[i] -= acc;
      }
      wave_sync_lds();
    }
  }
  __syncthreads();
  for (int k = t; k < n; k += 256) d.ycam[W.row_base + k] = z[k];
  // candidate cameras x + D^-1 delta (into x_pose[cur ^ 1]) and their rotation states
  {
    const int cur = d.st[w].cur;
    for (int ci = t; ci < W.n_poses; ci += 256) {
      const int c = W.pose_base + ci;
      double xn[6];
#pragma unroll
      for (int k = 0; k < 6; ++k) {
        xn[k] = d.x_pose[cur][6 * c + k] + (-z[6 * ci + k]) * d.scale_pose[6 * c + k];
        d.x_pose[cur ^ 1][6 * c + k] = xn[k];
      }
      d.rot_cand[c] = lorb::rot_val(xn);
    }
  }
#ifdef LORB_CHOL_STAMPS
  if (t == 0) { d.dbg[8 * w + 3] = __builtin_amdgcn_s_memtime() - T0 - d.dbg[8*w] - d.dbg[8*w+1] - d.dbg[8*w+2]; }
#endif
}

// K6w: banded Cholesky for band <= 48 on ONE wavefront per window, no workgroup barrier.
// The active 64 x 64 trailing window (rows/cols kb .. kb+63) lives in registers as ten 16 x 16
// tiles (I, J), J <= I < 4, in the v_mfma_f64_16x16x4f64 accumulator layout (register r of
// lane l: row 4r + (l >> 4), column l & 15).  Per 16-column panel:
//   1. the panel tiles (I, 0) go through a 64 x 17 LDS exchange to lane = row layout;
//   2. the 64 x 16 panel is factored in registers (v_readlane pivots, rsqrt + Newton, the
//      forward substitution fused);
//   3. L is stored into the LDS band (for the back-substitution) and re-read as MFMA operands
//      (A and B fragments of a tile are the same registers: B = L_J^T);
//   4. the rank-16 trailing update of tiles (I, J >= 1) runs as 24 MFMAs;
//   5. the window slides by 16: tiles move up-left, and the new bottom tile row comes straight
//      from S, because no earlier panel reaches it (L(i, k) = 0 for i - k > bw <= 48).
// Rows n .. n16-1 are an identity pad, so every panel is full; the next bottom tile row is
// prefetched one panel ahead.
__device__ __forceinline__ constexpr int tri4(int I, int J) { return I * (I + 1) / 2 + J; }

__global__ __launch_bounds__(256) void k_ba_chol_w(BaDev d) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int w = blockIdx.x;
  if (d.st[w].done) return;
  if (d.sharded && d.wfail[w] > 0.0) {  // a rank's point block was not PD: the step is invalid
    if (threadIdx.x == 0) d.st[w].chol_fail = 1;
    return;
  }
  const BaWin W = d.win[w];
  const int n = W.n, bw = W.bw;
  const int n16 = (n + 15) & ~15;
  const int t = threadIdx.x, lane = t & 63, ci = lane & 15, ck = lane >> 4;
  double* A = smem;                          // S band, overwritten in place by L: n16 x (bw + 1)
  double* z = A + (size_t)n16 * (bw + 1);    // rhs, overwritten by the forward substitution
  double* invd = z + n16;                    // n16
  double* xch = invd + n16;                  // 64 x 17 exchange
  const int dummy = (int)(xch + 64 * 17 + lane - A);  // 64 per-lane dummy slots after xch
  {  // stage S (+ identity pad rows) and rhs with all four waves, then wave 0 works alone
    const double* __restrict__ S = d.env + W.env_base;
    const int ne = n * (bw + 1);
    for (int k = t; k < ne; k += 256) A[k] = S[k];
    for (int k = ne + t; k < n16 * (bw + 1); k += 256) A[k] = (k % (bw + 1)) == bw ? 1.0 : 0.0;
    for (int k = t; k < n16; k += 256) z[k] = k < n ? d.rhs[W.row_base + k] : 0.0;
  }
  __syncthreads();
  if (t >= 64) return;
#ifdef LORB_CHOL_STAMPS
  unsigned long long T0 = __builtin_amdgcn_s_memtime(), tq = T0, ph[5] = {0, 0, 0, 0, 0};
#define CW_STAMP(k) do { const unsigned long long q_ = __builtin_amdgcn_s_memtime(); ph[k] += q_ - tq; tq = q_; } while (0)
#else
#define CW_STAMP(k) do {} while (0)
#endif
  auto sget = [&](int i, int j) -> double {  // band entry (i, j) of the staged matrix; branch-free
    const bool ok = j <= i && i - j <= bw && i < n16;
    const double v = A[ok ? i * (bw + 1) + (j - i + bw) : 0];
    return ok ? v : 0.0;
  };
  v4d T[10], Tn[4];
#pragma unroll
  for (int I = 0; I < 4; ++I)
#pragma unroll
    for (int J = 0; J <= I; ++J)
#pragma unroll
      for (int r = 0; r < 4; ++r) T[tri4(I, J)][r] = sget(16 * I + ck + 4 * r, 16 * J + ci);
  double zr = z[lane];
  bool bad = false;
  for (int kb = 0; kb < n16; kb += 16) {
    // the tile row that enters at the end of this panel (rows kb+64 .. kb+79): untouched S
#pragma unroll
    for (int J = 0; J < 4; ++J)
#pragma unroll
      for (int r = 0; r < 4; ++r) Tn[J][r] = sget(kb + 64 + ck + 4 * r, kb + 16 + 16 * J + ci);
    const double zin = kb + 16 + lane < n16 ? z[kb + 16 + lane] : 0.0;  // used by lanes >= 48
    // 1. panel tiles -> lane = row
#pragma unroll
    for (int I = 0; I < 4; ++I)
#pragma unroll
      for (int r = 0; r < 4; ++r) xch[(16 * I + ck + 4 * r) * 17 + ci] = T[tri4(I, 0)][r];
    wave_sync_lds();
    double P[NB];
#pragma unroll
    for (int q = 0; q < NB; ++q) P[q] = xch[lane * 17 + q];
    wave_sync_lds();
    CW_STAMP(0);
    // 2. factor the panel (lane = row kb + lane; entries above the diagonal are never stored)
    double yq = 0.0;
#pragma unroll
    for (int q = 0; q < NB; ++q) {
      const double akk = readlane_d(P[q], q);
      bad |= !(akk > 0.0);
      const double y = rsqrt_refined(akk);
      P[q] *= y;  // lane q: akk * y = L(k, k)
      yq = lane == q ? y : yq;
      const double zk = readlane_d(zr, q) * y;
      zr = lane > q ? fma(-P[q], zk, zr) : (lane == q ? zk : zr);
#pragma unroll
      for (int q2 = q + 1; q2 < NB; ++q2) {
        const double l = readlane_d(P[q], q2);
        P[q2] = fma(-P[q], l, P[q2]);
      }
    }
    CW_STAMP(1);
    // 3. L into the band (rows kb .. kb+63 have left S's use) + exchange; final z of the panel
    {
      const int row = kb + lane;
#pragma unroll
      for (int q = 0; q < NB; ++q) {
        const int col = kb + q;
        // branch-free: entries outside the band / above the diagonal go to a per-lane dummy slot
        const bool ok = row < n16 && col <= row && row - col <= bw;
        A[ok ? row * (bw + 1) + (col - row + bw) : dummy] = P[q];
        xch[lane * 17 + q] = P[q];
      }
      if (lane < NB) { z[row] = zr; invd[row] = yq; }
    }
    wave_sync_lds();
    double opA[4][4];  // [I][kk] = L(kb + 16 I + ci, kb + 4 kk + ck), I >= 1
#pragma unroll
    for (int I = 1; I < 4; ++I)
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) opA[I][kk] = xch[(16 * I + ci) * 17 + 4 * kk + ck];
    CW_STAMP(2);
    // 4. rank-16 trailing update (J = 1 first: it is the next panel)
#pragma unroll
    for (int J = 1; J < 4; ++J)
#pragma unroll
      for (int I = J; I < 4; ++I)
#pragma unroll
        for (int kk = 0; kk < 4; ++kk)
          T[tri4(I, J)] = __builtin_amdgcn_mfma_f64_16x16x4f64(-opA[I][kk], opA[J][kk], T[tri4(I, J)], 0, 0, 0);
    // 5. slide the window by 16 rows / columns
    {
      const double zs = __shfl_down(zr, 16, 64);  // rows kb+16 .. kb+63 move up
      zr = lane < 48 ? zs : zin;                  // rows kb+64 .. kb+79 enter (raw rhs)
    }
    T[tri4(0, 0)] = T[tri4(1, 1)];
    T[tri4(1, 0)] = T[tri4(2, 1)]; T[tri4(1, 1)] = T[tri4(2, 2)];
    T[tri4(2, 0)] = T[tri4(3, 1)]; T[tri4(2, 1)] = T[tri4(3, 2)]; T[tri4(2, 2)] = T[tri4(3, 3)];
#pragma unroll
    for (int J = 0; J < 4; ++J) T[tri4(3, J)] = Tn[J];
    CW_STAMP(3);
  }
  if (bad) {
#ifdef LORB_CHOL_STAMPS
    if (lane == 0) for (int k = 0; k < 5; ++k) d.dbg[8 * w + k] = ph[k];
#endif
    if (lane == 0) d.st[w].chol_fail = 1;
    return;
  }
  wave_sync_lds();
  // back substitution L^T y = z by 16-row blocks from the bottom.  Lane (g, j) = (lane >> 4,
  // lane & 15): the block's column j gathers sum_i L(i, j) y_i over the rows below (split over
  // the four lane groups, butterfly-reduced), then the 16 x 16 triangle is solved with
  // v_readlane broadcasts.
  {
    const int jc = lane & 15, g = lane >> 4;
    for (int c0 = n16 - 16; c0 >= 0; c0 -= 16) {
      const int j = c0 + jc;
      double lk[NB];
#pragma unroll
      for (int k = 0; k < NB; ++k) {  // L(c0 + k, j), k > jc, inside the band (bw < 15: not all of them)
        const bool ok = k > jc && k - jc <= bw;
        const double v = A[ok ? (c0 + k) * (bw + 1) + (j - (c0 + k) + bw) : 0];
        lk[k] = ok ? v : 0.0;
      }
      // rows i = c0+16+g+4u (u < 16) cover every row below the block that reaches column j
      // (i - j <= bw <= 48); all loads are issued before the FMAs, four independent chains
      const int iend = min(n16 - 1, j + bw);
      double av[16], zv[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int i = c0 + 16 + g + 4 * u;
        const bool ok = i <= iend;
        av[u] = A[ok ? i * (bw + 1) + (j - i + bw) : 0];
        zv[u] = z[ok ? i : 0];
        av[u] = ok ? av[u] : 0.0;
      }
      double a4[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int u = 0; u < 16; ++u) a4[u & 3] = fma(av[u], zv[u], a4[u & 3]);
      double acc = (a4[0] + a4[1]) + (a4[2] + a4[3]);
      {  // butterfly xor 16, xor 32 (permlane swaps, no LDS)
        double a, b;
        xrow_pair<false>(acc, a, b); acc = a + b;
        xrow_pair<true>(acc, a, b); acc = a + b;
      }
      double zb = z[j] - acc;
      const double iv = invd[j];
#pragma unroll
      for (int k = NB - 1; k >= 0; --k) {
        const double yk = readlane_d(zb, k) * readlane_d(iv, k);
        zb = jc == k ? yk : fma(-lk[k], yk, zb);
      }
      if (g == 0) z[j] = zb;
      wave_sync_lds();
    }
  }
  CW_STAMP(4);
#ifdef LORB_CHOL_STAMPS
  if (lane == 0) for (int k = 0; k < 5; ++k) d.dbg[8 * w + k] = ph[k];
#endif
#undef CW_STAMP
  for (int k = lane; k < n; k += 64) d.ycam[W.row_base + k] = z[k];
  const int cur = d.st[w].cur;
  for (int ci2 = lane; ci2 < W.n_poses; ci2 += 64) {
    const int c = W.pose_base + ci2;
    double xn[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      xn[k] = d.x_pose[cur][6 * c + k] + (-z[6 * ci2 + k]) * d.scale_pose[6 * c + k];
      d.x_pose[cur ^ 1][6 * c + k] = xn[k];
    }
    d.rot_cand[c] = lorb::rot_val(xn);
  }
}

// K6t: two-sided ("twisted") banded Cholesky for band <= 48 and n >= 128.  The chain of
// dependent panels is the cost of K6w (one wavefront is latency/issue bound), so the matrix is
// split into T = [0, m), M = [m, m+48) and B = [m+48, n16): T and B do not couple (band <= 48).
// Wave 0 eliminates T top-down and wave 1 eliminates B bottom-up concurrently: the bottom part
// is staged REVERSED (row i' = n16-1-i; the band of the reversed matrix is the same), so both
// waves run the identical panel code on their own LDS band.  Their windows end on M holding
// S_MM - L_MT L_MT^T and S_MM - L_MB L_MB^T; wave 0 combines them (minus S_MM) and factors M
// (3 panels).  Back-substitution: M, then T (wave 0) and B (wave 1) concurrently.  Rows
// n .. n16-1 are an identity pad.
// Progressive staging (k_ba_chol_2s): bit b of the workgroup's mask = rows [16 b, 16 b + 16) of the
// band are in LDS.  Waves 2 / 3 publish with release, the factoring waves wait with acquire.
__device__ __forceinline__ void wait_bit(unsigned long long* mask, int b) {
  while (!((__hip_atomic_load(mask, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) >> b) & 1ull))
    __builtin_amdgcn_s_sleep(1);
}
// SLEEP: the waiting wave backs off between polls so that it does not compete for LDS with the
// chain it waits on; the chain wave's own wait is short and spins
template <bool SLEEP>
__device__ __forceinline__ void wait_ge(int* c, int v) {
  while (__hip_atomic_load(c, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < v)
    if (SLEEP) __builtin_amdgcn_s_sleep(1);
}

// 1: the update waves spin on the chain's L post instead of sleeping between polls (same-box A/B
// 46.2 / 46.1 vs 46.1 / 45.5 us: inside the noise, off)
// Column stride of the chain's L columns in xch, padded against bank conflicts when the update
// wave reads them in MFMA operand layout.
constexpr int kCS = 65;
struct BandSide {
  double* A;     // band storage of the whole matrix (row-major, rows x (bw + 1), row i holds cols
                 // i-bw .. i); the diagonal slot holds 1 / L(i, i) (its only use is the
                 // back-substitution).  Element (i, j) of this side's view is A[base + si*i + sj*j]:
                 // the top side views it as is (si = bw, sj = 1, base = bw); the bottom side views
                 // it reversed, (i', j') = (n16-1-j, n16-1-i) (si = -1, sj = -bw, base =
                 // (n16-1)(bw+1) + bw), so both sides run the same panel code on one staging.
  double* z;     // rows: rhs -> forward substitution -> solution
  double* xch;   // 64 x 17 exchange (column 16 of each row: dummy store slot of that lane)
  int rows, bw, lane;
  int base, si, sj;
  unsigned long long* mask = nullptr;  // progressive staging (null: the whole band is staged)
  int* pdone = nullptr;                // panels whose L is in the band (release-counted, for linv)
  int nbk = 0, dir = 0;                // row blocks; +1 top view, -1 reversed bottom view
  int zslot = 0;                       // A[zslot] == 0.0 (out-of-band reads of the back-substitution)
  double* kco = nullptr;               // this side's back-substitution operators (bsk_block)
  unsigned long long* phases = nullptr;  // LORB_CHOL_PHASES diagnostics: chain wait / factor / store cycles
  unsigned long long* trace = nullptr;   // LORB_CHOL_TRACE diagnostics: per-panel event times
  int tslot = 0;                         // (slot of this wave's next panel; cycles since t0)
  int bslot = 320;                       // (slot of this wave's next back-substitution block)
  unsigned long long t0 = 0;
  __device__ __forceinline__ void tr(int k) const {
#ifdef LORB_CHOL_TRACE
    if (trace && lane == 0) trace[tslot + k] = __builtin_amdgcn_s_memtime() - t0;
#endif
  }

  __device__ __forceinline__ int idx(int i, int j) const { return base + si * i + sj * j; }

  __device__ __forceinline__ double get(int i, int j) const {  // branch-free; 0 outside band / rows
    const bool ok = j <= i && i - j <= bw && i < rows;
    const double v = A[ok ? idx(i, j) : base];
    return ok ? v : 0.0;
  }
  __device__ __forceinline__ void init_tiles(v4d (&T)[10]) const {  // column 0 is the chain wave's
#pragma unroll
    for (int I = 1; I < 4; ++I)
#pragma unroll
      for (int J = 1; J <= I; ++J)
#pragma unroll
        for (int r = 0; r < 4; ++r) T[tri4(I, J)][r] = get(16 * I + (lane >> 4) + 4 * r, 16 * J + (lane & 15));
  }
  __device__ __forceinline__ void init_panel(double (&P)[NB], double& zr) const {
#pragma unroll
    for (int q = 0; q < NB; ++q) P[q] = get(lane, q);
    zr = lane < rows ? z[lane] : 0.0;
  }
  // Lookahead split of the panel loop over two wavefronts of one side.  The CHAIN wave factors
  // panels kb = kb0, kb0+16, ... < kend (lane = panel row): v_readlane pivots, rsqrt-refined, the
  // forward substitution fused; it writes L to the band and to xch and posts *lrd.  The UPDATE
  // wave holds the 64 x 64 trailing window as ten 16 x 16 MFMA accumulator tiles: on each posted
  // panel it first applies the rank-16 update to the next panel's column (tiles (1..3, 1)), hands
  // that column to the chain wave through pb (lane = row) and posts *prd, and only then updates
  // the rest of the window and slides it by 16 -- off the chain's critical path.
  //   chain(): P = the first panel when `pre` (else it comes from pb); pwant counts the pb posts
  //   consumed so far (continues across phases).
  __device__ __forceinline__ void chain(double (&P)[NB], double& zr, bool& bad, int kb0, int kend, bool pre,
                                        int* lrd, int* prd, int& pwant, const double* pb) const {
    const int dstep = 16 * (si + sj);  // address step of one panel along the diagonal
    unsigned l_ok = 0;
#pragma unroll
    for (int q = 0; q < NB; ++q) l_ok |= (unsigned)(q <= lane && lane - q <= bw) << q;
    int l_base = idx(kb0 + lane, kb0);  // slot of (kb0 + lane, kb0 + q) = l_base + q sj
    // L column q of the panel at colbuf[q * kCS + row]: the chain's multipliers and what the
    // update wave reads (in MFMA operand layout)
    double* colbuf = xch;
    // dummy target of the masked band stores (outside colbuf)
    double* dummy = xch + 16 * kCS + lane;
#ifdef LORB_CHOL_PHASES
    unsigned long long ph_w = 0, ph_c = 0, ph_s = 0, tq = __builtin_amdgcn_s_memtime();
#define CH_PH(v) do { const unsigned long long q_ = __builtin_amdgcn_s_memtime(); v += q_ - tq; tq = q_; } while (0)
#else
#define CH_PH(v) do {} while (0)
#endif
    for (int kb = kb0; kb < kend; kb += 16) {
      // Opaque per-iteration copies of the lane constants: otherwise every lane comparison of the
      // unrolled panel is hoisted out of the loop as an SGPR mask and the masks spill.
      int lane = this->lane, lok = (int)l_ok;
      asm volatile("" : "+v"(lane), "+v"(lok));
      if (!(pre && kb == kb0)) {
        wait_ge<false>(prd, ++pwant);
#pragma unroll
        for (int q = 0; q < NB; ++q) P[q] = pb[lane * 17 + q];  // lanes < q: upper garbage, never used
      }
      CH_PH(ph_w);
      tr(0);
      const double zin = kb + 16 + lane < rows ? z[kb + 16 + lane] : 0.0;
      double yq = 0.0;
      // Software-pipelined columns: column q-1's updates of the later columns (multipliers loaded
      // from colbuf at the end of iteration q-1) are issued inside column q's pivot chain, behind
      // a scheduling barrier after the first Newton step of its rsqrt, so the chain no longer
      // waits on LDS.  Every P[q2] still receives its FMAs in column order (same bits).
      double mp[NB];
#pragma unroll
      for (int q2 = 0; q2 < NB; ++q2) mp[q2] = 0.0;
      double akk = readlane_d(P[0], 0);
#pragma unroll
      for (int q = 0; q < NB; ++q) {
        bad |= !(akk > 0.0);
        double y = __builtin_amdgcn_rsq(akk);
        __builtin_amdgcn_sched_barrier(0);
        if (q >= 1) {
#pragma unroll
          for (int q2 = q + 1; q2 < NB; ++q2) P[q2] = fma(-P[q - 1], mp[q2], P[q2]);
        }
        // The chain wave is VALU-issue bound (about 45 instructions per column): one Newton step on
        // v_rsq_f64 (about 2^-23 relative) leaves ~1e-14, far inside north_star's 1e-5
        {
          const double e = fma(-akk * y, y, 1.0);
          y = fma(0.5 * y, e, y);
        }
        P[q] *= y;  // lane q: akk * y = L(k, k)
        yq = lane == q ? y : yq;
        const double zk = readlane_d(zr, q) * y;
        zr = lane > q ? fma(-P[q], zk, zr) : (lane == q ? zk : zr);
        colbuf[q * kCS + lane] = P[q];
        if (q + 1 < NB) {
          const double l1 = readlane_d(P[q], q + 1);
          P[q + 1] = fma(-P[q], l1, P[q + 1]);
          akk = readlane_d(P[q + 1], q + 1);
#pragma unroll
          for (int q2 = q + 2; q2 < NB; ++q2) mp[q2] = colbuf[q * kCS + q2];
        }
      }
      CH_PH(ph_c);
      tr(1);
      const bool rowvalid = kb + lane < rows;
      // the update wave reads L from colbuf: post it now, then store L to the band (for the
      // diagonal-block inverses and the back-substitution) while the update runs
      if (lane == 0) __hip_atomic_fetch_add(lrd, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
#pragma unroll
      for (int q = 0; q < NB; ++q) {
        const bool ok = rowvalid && (((unsigned)lok >> q) & 1u);
        *(ok ? A + l_base + q * sj : dummy) = q == lane ? yq : P[q];
      }
      l_base += dstep;
      if (lane < NB) z[kb + lane] = zr;
      if (lane == 0 && pdone) __hip_atomic_fetch_add(pdone, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      const double zs = __shfl_down(zr, 16, 64);
      zr = lane < 48 ? zs : zin;
      CH_PH(ph_s);
      tr(2);
      const_cast<BandSide*>(this)->tslot += 3;
    }
#ifdef LORB_CHOL_PHASES
    if (phases && this->lane == 0) { phases[0] += ph_w; phases[1] += ph_c; phases[2] += ph_s; }
#endif
#undef CH_PH
  }
  //   update(): T = the window at kb0 (column 0 unused); on return the window at kend (all ten
  //   tiles).  lwant counts the L posts consumed so far.
  __device__ __forceinline__ void update(v4d (&T)[10], int kb0, int kend, int* lrd, int* prd, int& lwant,
                                         double* pb) const {
    const int ci = lane & 15, ck = lane >> 4;
    const int dstep = 16 * (si + sj);
    int tn_addr = idx(kb0 + 64 + ck, kb0 + 16 + ci);  // entering tile (J, r) adds 4 r si + 16 J sj (below)
    unsigned tn_ok = 0;
#pragma unroll
    for (int J = 0; J < 4; ++J)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = 64 + ck + 4 * r, j = 16 + 16 * J + ci;
        tn_ok |= (unsigned)(j <= i && i - j <= bw) << (4 * J + r);
      }
    for (int kb = kb0; kb < kend; kb += 16) {
      int tok = (int)tn_ok;
      asm volatile("" : "+v"(tok));
      // the tile row entering at the end of this panel (view rows kb+64 .. kb+79): untouched S,
      // loaded while the chain wave factors the panel
      if (mask) {
        const int b = dir > 0 ? kb / 16 + 4 : nbk - 5 - kb / 16;
        if (b >= 0 && b < nbk) wait_bit(mask, b);
      }
      v4d Tn[4];
#pragma unroll
      for (int J = 0; J < 4; ++J)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          // (kb+64+ck+4r, kb+16+16J+ci): row offset 4r, column offset 16J relative to tn_addr
          const bool ok = (((unsigned)tok >> (4 * J + r)) & 1u) && kb + 64 + ck + 4 * r < rows;
          const double v = A[ok ? tn_addr + 4 * r * si + 16 * J * sj : base];
          Tn[J][r] = ok ? v : 0.0;
        }
      tn_addr += dstep;
      const bool nxt = kb + 16 < kend;
      tr(0);
      wait_ge<true>(lrd, ++lwant);
      tr(1);
      double opA[4][4];
#pragma unroll
      for (int I = 1; I < 4; ++I)
#pragma unroll
        for (int kk = 0; kk < 4; ++kk)
          opA[I][kk] = xch[(4 * kk + ck) * kCS + 16 * I + ci];  // L(kb + 16 I + ci, kb + 4 kk + ck)
      // the next panel's column first, then hand it over
#pragma unroll
      for (int kk = 0; kk < 4; ++kk)
#pragma unroll
        for (int I = 1; I < 4; ++I)
          T[tri4(I, 1)] = __builtin_amdgcn_mfma_f64_16x16x4f64(-opA[I][kk], opA[1][kk], T[tri4(I, 1)], 0, 0, 0);
      if (nxt) {
#pragma unroll
        for (int I = 1; I < 4; ++I)
#pragma unroll
          for (int r = 0; r < 4; ++r) pb[(16 * (I - 1) + ck + 4 * r) * 17 + ci] = T[tri4(I, 1)][r];
#pragma unroll
        for (int r = 0; r < 4; ++r) pb[(48 + ck + 4 * r) * 17 + ci] = Tn[0][r];
        if (lane == 0) __hip_atomic_fetch_add(prd, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      tr(2);
      // k-step outer: the three tiles' accumulation chains interleave
#pragma unroll
      for (int kk = 0; kk < 4; ++kk)
#pragma unroll
        for (int J = 2; J < 4; ++J)
#pragma unroll
          for (int I = J; I < 4; ++I)
            T[tri4(I, J)] = __builtin_amdgcn_mfma_f64_16x16x4f64(-opA[I][kk], opA[J][kk], T[tri4(I, J)], 0, 0, 0);
      T[tri4(0, 0)] = T[tri4(1, 1)];
      T[tri4(1, 0)] = T[tri4(2, 1)]; T[tri4(1, 1)] = T[tri4(2, 2)];
      T[tri4(2, 0)] = T[tri4(3, 1)]; T[tri4(2, 1)] = T[tri4(3, 2)]; T[tri4(2, 2)] = T[tri4(3, 3)];
#pragma unroll
      for (int J = 0; J < 4; ++J) T[tri4(3, J)] = Tn[J];
      tr(3);
      const_cast<BandSide*>(this)->tslot += 4;
    }
  }
  // The 16 x 16 diagonal block of L at view rows c0 .. c0+15 replaced in place by its inverse X
  // (lower triangular; the diagonal slot already holds 1 / L(i, i) = X(i, i)):
  // X(i, j) = -X(i, i) sum_{k=j}^{i-1} L(i, k) X(k, j).  Only the back-substitution reads the
  // block afterwards.  All 64 lanes: lane = 4 j + r holds column j's rows i = 4 m + r (acc[m]).  Step k: the lane
  // of row k (r = k & 3) forms X(k, j) and stores it, a quad broadcast hands it to the column's
  // four lanes, each adds L(i, k) X(k, j) to its rows.  The L loads (about 30 per lane) are all
  // issued before the sweep.  Per row the FMAs run in k order (the bits of a column sweep).
  template <int K>
  __device__ __forceinline__ void linv_step(int c0, int j, int r, double (&acc)[4], const double (&dv)[4],
                                            const double (&lv)[16][4]) const {
    constexpr int rk = K & 3, mk = K >> 2;
    const double xo = K == j ? dv[mk] : (K > j ? -dv[mk] * acc[mk] : 0.0);
    if (r == rk && K > j && K - j <= bw) A[idx(c0 + K, c0 + j)] = xo;
    const double xk = dpp_d<rk * 0x55>(xo);
#pragma unroll
    for (int m = 0; m < 4; ++m)
      if (4 * m + 3 > K) acc[m] = fma(lv[K][m], xk, acc[m]);  // lv == 0 where 4 m + r <= K
  }
  template <int K>
  __device__ __forceinline__ void linv_sweep(int c0, int j, int r, double (&acc)[4], const double (&dv)[4],
                                             const double (&lv)[16][4]) const {
    linv_step<K>(c0, j, r, acc, dv, lv);
    if constexpr (K + 1 < 16) linv_sweep<K + 1>(c0, j, r, acc, dv, lv);
  }
  __device__ __forceinline__ void linv(int c0) const {
    const int j = lane >> 2, r = lane & 3;
    double acc[4] = {0.0, 0.0, 0.0, 0.0}, dv[4], lv[16][4];
#pragma unroll
    for (int m = 0; m < 4; ++m) dv[m] = A[idx(c0 + 4 * m + r, c0 + 4 * m + r)];
#pragma unroll
    for (int k = 0; k < 16; ++k)
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        if (4 * m + 3 > k) {
          const int i = 4 * m + r;
          lv[k][m] = A[(i > k && i - k <= bw) ? idx(c0 + i, c0 + k) : zslot];
        } else {
          lv[k][m] = 0.0;
        }
      }
    linv_sweep<0>(c0, j, r, acc, dv, lv);
  }
  // Back-substitution L^T y = z, push style: the 64 rows c0-48 .. c0+15 of the current block c0
  // live in registers (row r in lane r & 63, so sliding the window needs no shuffle).  A block
  // solves its 16 x 16 triangle -- as a v_readlane chain (c0 >= c_inv) or as one product with the
  // inverted diagonal block X from linv (c0 < c_inv) -- writes y to z, pushes y into the rows above
  // it within the band, and its lanes load the rows that enter the window above.
  __device__ __forceinline__ int bs_row(int c0) const { return c0 - 48 + ((lane - (c0 - 48)) & 63); }
  // window of block c_hi; `known` rows c_hi+16 .. c_hi+15+known already hold final y in z and are
  // pushed into it first
  __device__ __forceinline__ double bs_init(int c_hi, int known) const {
    const int row = bs_row(c_hi);
    double zw = row >= 0 ? z[row] : 0.0;
    for (int i0 = 0; i0 < known; i0 += 16) {
      double l[16], y[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int ri = c_hi + 16 + i0 + k;
        const bool ok = i0 + k < known && row >= 0 && ri - row <= bw;
        l[k] = A[ok ? idx(ri, row) : base];
        l[k] = ok ? l[k] : 0.0;
        y[k] = z[i0 + k < known ? ri : 0];
      }
#pragma unroll
      for (int k = 0; k < 16; ++k) zw = fma(-l[k], y[k], zw);
    }
    return zw;
  }
  struct BsWin {
    double zw;         // the window
    double zin = 0.0;  // rows that entered above (loaded by the last block's lanes), merged late
    bool pend = false;
  };
  // blocks c_from, c_from - 16, ..., c_to; INV: multiply by the inverted diagonal block, else a
  // v_readlane chain through the triangle.  The rows entering above are merged only before the
  // next block's pushes, so their loads are off the chain.  Addresses are per-lane linear in the
  // block index; the lane constants are kept opaque (VGPRs) so the unrolled block does not
  // hoist dozens of uniform values into SGPRs.
  template <bool INV>
  __device__ __forceinline__ void bs_run(BsWin& S, int c_from, int c_to) const {
    for (int c0 = c_from; c0 >= c_to; c0 -= 16) {
      int row = bs_row(c0);
      const int j = row - c0, b0 = c0 & 63;
      const bool blk = j >= 0;
      // L(c0 + k, row) at aL + si k, valid for 1 <= c0 - row + k <= bw (and row >= 0; INV: not a
      // block lane); X(c0 + k, c0 + j) at aX + si k, valid for k >= j.  Invalid entries read the
      // zero word, so a load needs one compare and one address select.
      int aL = base + si * c0 + sj * row;
      int aX = base + si * c0 + sj * (c0 + j);
      int eL = c0 - row - 1 + ((row < 0 || (INV && blk)) ? (1 << 20) : 0);
      int eX = blk ? -j : (1 << 20);
      asm volatile("" : "+v"(aL), "+v"(aX), "+v"(eL), "+v"(eX), "+v"(row));
      double Lp[16], xv[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) Lp[k] = A[(unsigned)(eL + k) < (unsigned)bw ? aL + si * k : zslot];
      double zw = S.zw;
      if (!INV) {
#pragma unroll
        for (int k = 0; k < 16; ++k) xv[k] = A[base + si * (c0 + k) + sj * (c0 + k)];  // 1 / L(i, i)
        zw = S.pend ? S.zin : zw;
#pragma unroll
        for (int k = 15; k >= 0; --k) {
          const double yk = readlane_d(zw, (b0 + k) & 63) * xv[k];
          zw = (j == k) ? yk : fma(-Lp[k], yk, zw);
        }
        if (blk) z[row] = zw;
      } else {
#pragma unroll
        for (int k = 0; k < 16; ++k) xv[k] = A[(unsigned)(eX + k) < 16u ? aX + si * k : zslot];
        // z_b and then y_b go through z in LDS (broadcast reads)
        if (blk) z[row] = zw;
        wave_sync_lds();
        double a4[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int k = 0; k < 16; ++k) a4[k & 3] = fma(xv[k], z[c0 + k], a4[k & 3]);
        const double y = (a4[0] + a4[1]) + (a4[2] + a4[3]);
        wave_sync_lds();
        if (blk) z[row] = y;
        wave_sync_lds();
        zw = S.pend ? S.zin : zw;
        double p4[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int k = 0; k < 16; ++k) p4[k & 3] = fma(Lp[k], z[c0 + k], p4[k & 3]);
        zw = blk ? y : zw - ((p4[0] + p4[1]) + (p4[2] + p4[3]));
      }
      if (blk) S.zin = row - 64 >= 0 ? z[row - 64] : 0.0;  // the row entering above
      S.pend = blk;
      S.zw = zw;
    }
  }
  // Back-substitution operator of T / B block c0, built off the critical path (after the block's
  // diagonal inverse X): the block's step -- y = X^T z_b, then the push of y into the 47 rows
  // above -- folded into ONE product with z_b.  Lane l (window row r = bs_row(c0)) gets
  //   block rows (j = r - c0 >= 0):  coef[k] = X(k, j)                          (y_j = sum_k coef[k] z_k)
  //   rows above:                    coef[k] = sum_{j <= k} L(c0 + j, r) X(k, j) (zw_r -= sum_k coef[k] z_k)
  // at kco[(c0 / 16) * 1024 + 64 k + l].  The bs_run_k step is then one LDS round trip (publish z_b,
  // 16 broadcast reads) where bs_run<true> has two.  X is the full 16 x 16 block: bw >= 15.
  // On the matrix cores: C(k, r) = sum_j X(k, j) Lx(j, r), rows r = c0-48 .. c0+15 as four 16-row
  // tiles (N), j in four steps of 4 (K), 16 v_mfma_f64_16x16x4f64; Lx(j, r) = L(c0 + j, r) above the
  // block (0 outside the band / matrix) and the identity on the block's own rows.  Per lane 4 + 12
  // independent LDS loads (no broadcasts); C lands as kco[64 k + (r & 63)], the lane of row r in
  // bs_run_k's window.
  __device__ __forceinline__ void bsk_block(int c0) const {
    const int ci = lane & 15, ck = lane >> 4;
    double xa[4], lb[3][4];
#pragma unroll
    for (int st = 0; st < 4; ++st) {
      const int j = 4 * st + ck;  // A: X(ci, j), lower triangle
      xa[st] = A[j <= ci ? idx(c0 + ci, c0 + j) : zslot];
#pragma unroll
      for (int t = 0; t < 3; ++t) {  // B: L(c0 + j, r) for the rows above
        const int r = c0 - 48 + 16 * t + ci, dd = c0 + j - r;
        lb[t][st] = A[(r >= 0 && dd >= 1 && dd <= bw) ? idx(c0 + j, r) : zslot];
      }
    }
    v4d acc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = v4d{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int st = 0; st < 4; ++st) {
#pragma unroll
      for (int t = 0; t < 3; ++t) acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(xa[st], lb[t][st], acc[t], 0, 0, 0);
      const double id = (4 * st + ck) == ci ? 1.0 : 0.0;  // the block's rows: X(k, r - c0)
      acc[3] = __builtin_amdgcn_mfma_f64_16x16x4f64(xa[st], id, acc[3], 0, 0, 0);
    }
    double* o = kco + (c0 >> 4) * 1024;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int k = 4 * q + ck;  // coefficient pairs (k, k + 1) of a lane adjacent: 16-byte loads
        o[128 * (k >> 1) + 2 * ((c0 - 48 + 16 * t + ci) & 63) + (k & 1)] = acc[t][q];
      }
  }
  __device__ __forceinline__ void bsk_load(int c0, double (&cf)[16]) const {
    const double2* p = reinterpret_cast<const double2*>(kco + (c0 >> 4) * 1024) + lane;
#pragma unroll
    for (int k2 = 0; k2 < 8; ++k2) {
      const double2 v = p[64 * k2];
      cf[2 * k2] = v.x; cf[2 * k2 + 1] = v.y;
    }
  }
  // blocks c_from, c_from - 16, ..., c_to through their bsk_block operators; cf holds block
  // c_from's on entry.  Two coefficient sets alternate, so the next block's loads (L2) stay in
  // flight while this block runs (a copy between sets would wait for them).  Rows entering above
  // are merged before the product, as in bs_run.
  __device__ __forceinline__ void tr_bs(int k) const {  // LORB_CHOL_TRACE: back-substitution steps
#ifdef LORB_CHOL_TRACE
    if (trace && lane == 0 && bslot + k < 512) trace[bslot + k] = __builtin_amdgcn_s_memtime() - t0;
#endif
  }
  // cn: the next block's operator is requested into cg once z_b is published (the issue of its
  // loads overlaps the publish's round trip instead of sitting between two blocks)
  __device__ __forceinline__ void bsk_step(BsWin& S, int c0, const double (&cf)[16], int cn, double (&cg)[16]) const {
    tr_bs(0);
    int row = bs_row(c0);
    asm volatile("" : "+v"(row));
    const int j = row - c0;
    const bool blk = j >= 0;
    // branch-free: the other lanes' stores go to their dummy slot (xch column 16), their entering-
    // row load to the zero word (an exec-masked branch made the compiler wait for that load on the
    // chain right after the product)
    double* pub = blk ? z + row : xch + 17 * lane + 16;
    const double* ent = (blk && row >= 64) ? z + (row - 64) : A + zslot;
    double zw = S.zw;
    *pub = zw;  // z_b is final: publish it
    zw = S.pend ? S.zin : zw;
    const double zin = *ent;  // the row entering above (never pushed yet: off the chain)
    bsk_load(cn, cg);
    wave_sync_lds();
    tr_bs(1);
    const double2* zb2 = reinterpret_cast<const double2*>(z + c0);
    double a4[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int k2 = 0; k2 < 8; ++k2) {
      const double2 v = zb2[k2];
      a4[(2 * k2) & 3] = fma(cf[2 * k2], v.x, a4[(2 * k2) & 3]);
      a4[(2 * k2 + 1) & 3] = fma(cf[2 * k2 + 1], v.y, a4[(2 * k2 + 1) & 3]);
    }
    const double sum = (a4[0] + a4[1]) + (a4[2] + a4[3]);
    zw = blk ? sum : zw - sum;
    tr_bs(2);
    const_cast<BandSide*>(this)->bslot += 3;
    *pub = zw;  // y_b (after every lane's broadcast read: a wave's LDS operations stay in order)
    S.zin = zin;
    S.pend = blk;
    S.zw = zw;
  }
  // fully unrolled (at most kBskMax blocks): in a loop the compiler drains every load at the loop
  // head (vmcnt(0)), which would make each block wait for its successor's prefetch
  static constexpr int kBskMax = 32;
  __device__ __forceinline__ void bs_run_k(BsWin& S, int c_from, int c_to, double (&cf)[16]) const {
    double cg[16];
    int c0 = c_from;
#pragma unroll
    for (int it = 0; it < kBskMax; it += 2) {
      if (c0 < c_to) return;
      bsk_step(S, c0, cf, c0 - 16 >= c_to ? c0 - 16 : c0, cg);
      if (c0 - 16 < c_to) return;
      bsk_step(S, c0 - 16, cg, c0 - 32 >= c_to ? c0 - 32 : c0, cf);
      c0 -= 32;
    }
    for (; c0 >= c_to; c0 -= 16) {  // more than kBskMax blocks (narrow bands of ~1000 rows)
      bsk_step(S, c0, cf, c0 - 16 >= c_to ? c0 - 16 : c0, cg);
#pragma unroll
      for (int k = 0; k < 16; ++k) cf[k] = cg[k];
    }
  }
};

// Flat copy of band chunks [j0, j1) (16-byte chunks of the row-major n x (bw + 1) band) by nthr
// threads, U chunks per thread per batch with all loads of a batch issued before any store.
// Element (i, off) keeps S's value inside the matrix; the left triangle of the first bw rows is
// zeroed and rows n .. n16-1 are an identity pad.
template <int U>
__device__ __forceinline__ void stage_band(const double2* __restrict__ S2, double* Ab, int j0, int j1, int tid,
                                           int nthr, int n, int bw, int nsrc) {
  const int B1 = bw + 1;
  for (int jb = j0 + tid; jb < j1; jb += nthr * U) {
    double2 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int j = jb + nthr * u;
      v[u] = S2[(j < j1 && j < nsrc) ? j : 0];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int j = jb + nthr * u;
      if (j < j1) {
        int i = (2 * j) / B1, off = (2 * j) % B1;
        double e[2] = {v[u].x, v[u].y};
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const bool in = i < n && i - (bw - off) >= 0;
          e[h] = in ? e[h] : ((i >= n && off == bw) ? 1.0 : 0.0);
          if (++off == B1) { off = 0; ++i; }
        }
        reinterpret_cast<double2*>(Ab)[j] = double2{e[0], e[1]};
      }
    }
  }
}


// the fused iteration's camera-block terms (stage_fix's), added by the staging thread itself
// the same over two chunk ranges [a0, a1) and [b0, b1), all loads of a batch before any store;
template <int U>
__device__ __forceinline__ void stage_band2(const double2* __restrict__ S2, double* Ab, int a0, int a1, int b0, int b1,
                                            int tid, int nthr, int n, int bw, int nsrc) {
  const int B1 = bw + 1, la = a1 - a0, tot = la + (b1 - b0);
  for (int vb = tid; vb < tot; vb += nthr * U) {
    double2 v[U];
    int jj[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int vv = vb + nthr * u;
      jj[u] = vv < la ? a0 + vv : b0 + (vv - la);
      v[u] = S2[(vv < tot && jj[u] < nsrc) ? jj[u] : 0];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int j = jj[u];
      if (vb + nthr * u < tot) {
        int i = (2 * j) / B1, off = (2 * j) % B1;
        double e[2] = {v[u].x, v[u].y};
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const bool in = i < n && i - (bw - off) >= 0;
          e[h] = in ? e[h] : ((i >= n && off == bw) ? 1.0 : 0.0);
          if (++off == B1) { off = 0; ++i; }
        }
        reinterpret_cast<double2*>(Ab)[j] = double2{e[0], e[1]};
      }
    }
  }
}

// The fused iteration's camera blocks: k_ba_red<2> stages sc (U - A) sc^T on the diagonal camera
// blocks, so rows [r0, r1) of the staged band only get D^2 = clamp(U_ii sc_i^2) / radius on the
// diagonal.  Threads tid, tid + nthr, ... of the caller.
__device__ __forceinline__ void stage_fix(const BaDev& d, const LMOpt& o, double* Ab, const BaWin& W, double radius,
                                          int r0, int r1, int tid, int nthr) {
  r1 = min(r1, W.n);
  const int B1 = W.bw + 1;
  for (int q = tid; q < (r1 - r0) * 6; q += nthr) {
    const int i = r0 + q / 6, i6 = i % 6, j6 = q % 6;
    if (j6 != i6) continue;
    const int c = W.pose_base + i / 6;
    const double* sc = d.scale_pose + 6 * c;
    double v = d.U[21 * c + u21(i6, j6)] * sc[i6] * sc[j6];
    v = 0.0 + fmin(fmax(v, o.min_diag), o.max_diag) / radius;
    double& e = Ab[i * B1 + (j6 - i6 + W.bw)];
    e = e + v;
  }
}

// stage_fix's term for item q of rows [r0, r1) (one item per thread when (r1 - r0) * 6 <= the
// threads): its value, and in `at` the band word it is added to (-1: none).  Computed before the
// band copy, so its loads share the copy's round trip; the same expression, the same bits.
__device__ __forceinline__ double stage_fix_val(const BaDev& d, const LMOpt& o, const BaWin& W, double radius,
                                                int r0, int r1, int q, int& at) {
  r1 = min(r1, W.n);
  at = -1;
  if (q >= (r1 - r0) * 6) return 0.0;
  const int i = r0 + q / 6, i6 = i % 6, j6 = q % 6;
  if (j6 != i6) return 0.0;
  const int c = W.pose_base + i / 6;
  const double* sc = d.scale_pose + 6 * c;
  double v = d.U[21 * c + u21(i6, j6)] * sc[i6] * sc[j6];
  v = 0.0 + fmin(fmax(v, o.min_diag), o.max_diag) / radius;
  at = i * (W.bw + 1) + (j6 - i6 + W.bw);
  return v;
}

constexpr int kChol2sThreads = 512;
// The T / B back-substitution runs one LDS round trip per block (BandSide::bsk_block / bs_run_k).
// (Measured and removed: the epilogue's pose state loaded at the kernel's start, 232 -> 256 VGPRs,
// no gain; y_T / y_B as w - G y_M with G and w formed during the M phase, 115 k cycles against
// 97 k -- DESIGN §4.)

// LDS words of k_ba_chol_2s: band (n16 rows), both sides' rhs (n16 + 48), two 64 x 18 exchanges
// (together the 48 x 48 combine), zX (48), two 64 x 17 panel hand-off buffers, a zero word
__host__ __device__ constexpr int chol2s_words(int n16, int bw) {
  return n16 * (bw + 1) + (n16 + 48) + 2 * 64 * 18 + 48 + 2 * 64 * 17 + 2;
}

// Waves: 0 / 1 chain (top / bottom side), 2 / 3 their update waves, 4 / 5 the inverses of L's
// diagonal blocks (for the back-substitution), 6 / 7 the progressive staging of the band.
// HEAD (the fused iteration): wave 4 first runs the iteration head (lm_head, k_ba_lm_begin's work)
// while the first panels factor; a head that ends the solve leaves the candidate unwritten.
template <bool HEAD>
__device__ __forceinline__ void chol_2s_run(const BaDev& d, const LMOpt& o, const int w) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  __shared__ int s_bad;
  __shared__ int s_head_done;
#ifdef LORB_CHOL_STAMPS
  const unsigned long long st_entry = __builtin_amdgcn_s_memtime();
#endif

  // window, state and failure flag requested together (one round trip before the band copy)
  const BaWin W = d.win[w];
  const WinState S0 = d.st[w];
  const int done = S0.done;
  const double wfail = d.sharded ? d.wfail[w] : 0.0;
  if (done) return;
  if (wfail > 0.0) {  // a rank's point block was not PD: the step is invalid
    if (HEAD) {       // the fused sharded iteration's head still runs (it advances the iteration)
      if (threadIdx.x < 64) {
        const WinState S = lm_head<true>(d, o, w, threadIdx.x, S0, W);
        if (threadIdx.x == 0 && !S.done) d.st[w].chol_fail = 1;
      }
    } else if (threadIdx.x == 0) {
      d.st[w].chol_fail = 1;
    }
    return;
  }
#ifdef LORB_CHOL_TRACE
  if (threadIdx.x == 0) d.dbg[512 * w + 250] = __builtin_amdgcn_s_memtime();  // raw: state loaded
#endif
  constexpr int NT = kChol2sThreads;
  const int n = W.n, bw = W.bw, B1 = bw + 1;
  const int n16 = (n + 15) & ~15;
  const int m = 16 * ((n16 - 48) / 32);  // T = [0, m), M = [m, m+48), B = [m+48, n16)
  const int nB = n16 - m - 48;
  const int rt = m + 48, rb = nB + 48;    // rows of the top / reversed-bottom bands
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  double* Ab = smem;          // the whole band once, n16 rows (rows n .. n16-1: identity pad)
  double* zt = Ab + n16 * B1;
  double* zb = zt + rt;
  double* xt = zb + rb;       // 64 x 18 per side (rows of 17); both together hold X (48 x 48)
  double* xb = xt + 64 * 18;
  double* zX = xb + 64 * 18;  // 48
  double* pbt = zX + 48;      // 64 x 17 panel hand-off, top / bottom
  double* pbb = pbt + 64 * 17;
  double* zero = pbb + 64 * 17;  // one 0.0
  // Staging.  The rows each side's first panel reads (view rows 0 .. 79 of both sides) are copied
  // by all waves; the rest of the band by waves 6 / 7 while the chains run, in the order the
  // update waves need it (a block mask in LDS).  Waves 4 / 5 invert the diagonal 16 x 16 blocks
  // of L as the panels finish, for the back-substitution.
  __shared__ unsigned long long s_mask;
  __shared__ int s_pdone[2];
  __shared__ int s_linv[2];           // diagonal-block inverses done, per side
  __shared__ int s_lrd[2], s_prd[2];  // per side: L panels posted (chain), panel columns posted (update)
  __shared__ int s_hand[3];           // T / B -> M hand-over (below)
  __shared__ int s_kdone[2];          // operator builders done, per side
  const double2* __restrict__ S2 = reinterpret_cast<const double2*>(d.env + W.env_base);
  const int nch = n16 * B1 / 2, nsrc = n * B1 / 2;  // chunks (n is a multiple of 6: even)
  const int nbk = n16 / 16, ib = 4;
#ifndef LORB_CHOL_PROG
#define LORB_CHOL_PROG 1
#endif

  const bool prog = LORB_CHOL_PROG && nbk <= 64 && nbk > 2 * ib;
  const int cpb = 8 * B1;  // chunks per 16-row block
  // rhs loads issued before the band copy (one round trip for both), with the fused iteration's
  // camera-block terms of the rows staged first (16 ib rows per side: one item per thread), which
  // would otherwise cost a round trip after the copy.  The epilogue's poses go to waves 6 / 7
  // (camera t - 384), idle since their staging
  static_assert(16 * 4 * 6 <= kChol2sThreads, "one stage_fix item per thread");
  int fa0 = -1, fa1 = -1;
  double fv0 = 0.0, fv1 = 0.0;
  if (HEAD && prog) {
    fv0 = stage_fix_val(d, o, W, S0.radius, 0, 16 * ib, t, fa0);
    fv1 = stage_fix_val(d, o, W, S0.radius, 16 * (nbk - ib), n16, t, fa1);
  }
  const int cur = S0.cur, ep = t - (NT - 128);  // epilogue: camera ep (+ 128 k) of the window
  double rz;
  {
    const int row = t < rt ? t : n16 - 1 - (t - rt);
    rz = (t < rt + rb && row < n) ? d.rhs[W.row_base + row] : 0.0;
    // (the rhs is complete: k_ba_red writes (V - R) sc)
  }
  if (prog) {  // both sides' first ib blocks in one batch
    stage_band2<7>(S2, Ab, 0, ib * cpb, (nbk - ib) * cpb, nch, t, NT, n, bw, nsrc);
  } else {
    stage_band<14>(S2, Ab, 0, nch, t, NT, n, bw, nsrc);
  }
  if (t < rt) zt[t] = rz;
  else if (t < rt + rb) zb[t - rt] = rz;
  for (int k = t + NT; k < rt + rb; k += NT) {  // (n16 > 464 only)
    const int row = k < rt ? k : n16 - 1 - (k - rt);
    double v = row < n ? d.rhs[W.row_base + row] : 0.0;
    if (k < rt) zt[k] = v; else zb[k - rt] = v;
  }
  if (t == 0) {
    *zero = 0.0;
    s_bad = 0;
    s_head_done = 0;
    s_pdone[0] = 0; s_pdone[1] = 0;
    s_linv[0] = 0; s_linv[1] = 0;
    s_lrd[0] = 0; s_lrd[1] = 0; s_prd[0] = 0; s_prd[1] = 0;
    s_hand[0] = 0; s_hand[1] = 0; s_hand[2] = 0;
    s_kdone[0] = 0; s_kdone[1] = 0;
    unsigned long long msk = 0;
    for (int b = 0; b < nbk; ++b) msk |= (unsigned long long)(!prog || b < ib || b >= nbk - ib) << (b & 63);
    s_mask = msk;
  }
  __syncthreads();
  if (HEAD) {  // the camera blocks of the rows staged so far
    if (prog) {
      if (fa0 >= 0) Ab[fa0] = Ab[fa0] + fv0;
      if (fa1 >= 0) Ab[fa1] = Ab[fa1] + fv1;
    } else {
      stage_fix(d, o, Ab, W, S0.radius, 0, n16, t, NT);
    }
    __syncthreads();
  }
  BandSide top{Ab, zt, xt, rt, bw, lane, bw, bw, 1};
  BandSide bot{Ab, zb, xb, rb, bw, lane, (n16 - 1) * B1 + bw, -1, -bw};
  top.pdone = &s_pdone[0]; bot.pdone = &s_pdone[1];
  top.zslot = (int)(zero - Ab); bot.zslot = top.zslot;
  top.kco = d.kco + (size_t)((W.row_base >> 4) + w) * 1024;
  bot.kco = top.kco + (size_t)(m >> 4) * 1024;
  top.nbk = bot.nbk = nbk; top.dir = 1; bot.dir = -1;
  if (prog) { top.mask = &s_mask; bot.mask = &s_mask; }
#ifdef LORB_CHOL_TRACE
  // dbg[512 w + ...]: chain top 0.. (3 per panel), update top 64.. (4 per panel), chain bottom
  // 128.., update bottom 160.., single events 200.., diagonal-block inverses 256..
  const unsigned long long tr0 = __builtin_amdgcn_s_memtime();
  unsigned long long* trb = d.dbg + 512 * w;
  top.trace = trb; bot.trace = trb; top.t0 = tr0; bot.t0 = tr0;
  if (t == 0) trb[252] = tr0;  // raw
  top.tslot = wv == 0 ? 0 : 64; bot.tslot = wv == 1 ? 128 : 160;
  top.bslot = 320; bot.bslot = 400;
#define TR1(k) do { if (lane == 0) trb[200 + (k)] = __builtin_amdgcn_s_memtime() - tr0; } while (0)
#else
#define TR1(k) do {} while (0)
#endif
  const int side = wv & 1;                 // 0 top, 1 bottom
  const BandSide& me = side == 0 ? top : bot;
  double* pb = side == 0 ? pbt : pbb;
  int* lrd = &s_lrd[side];
  int* prd = &s_prd[side];
  int lwant = 0, pwant = 0;
  bool bad = false;
  double zr = 0.0;
  double P[NB];
  v4d T[10];
  // LORB_CHOL_STAMPS: dbg[0..5] = waves 0..5 done with the T / B phase, [6] wave 0 done with M,
  // [7] wave 0 done with the back-substitution (cycles from the end of the initial staging)
#if defined(LORB_CHOL_STAMPS) && !defined(LORB_CHOL_PHASES)
  const unsigned long long st0 = __builtin_amdgcn_s_memtime();
#define C2_STAMP(k) do { if (lane == 0) d.dbg[8 * w + (k)] = __builtin_amdgcn_s_memtime() - st0; } while (0)
#else
#define C2_STAMP(k) do {} while (0)
#endif
  if (wv >= 6) {
    if (prog) {  // remaining blocks [ib, nbk - ib): wave 6 from the top, wave 7 from the bottom
      const int lo = ib, hi = nbk - ib, mid = (lo + hi) / 2;
      for (int k = 0; k < (side == 0 ? mid - lo : hi - mid); ++k) {
        const int b = side == 0 ? lo + k : hi - 1 - k;
        stage_band<7>(S2, Ab, b * cpb, min((b + 1) * cpb, nch), lane, 64, n, bw, nsrc);
        if (HEAD) {
          wave_sync_lds();
          stage_fix(d, o, Ab, W, S0.radius, 16 * b, 16 * b + 16, lane, 64);
        }
        if (lane == 0) __hip_atomic_fetch_or(&s_mask, 1ull << b, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
    TR1(8 + side);
  }
  if (HEAD && wv == 4) {  // the iteration head while the first panels factor
    const WinState S = d.sharded ? lm_head<true>(d, o, w, lane, S0, W) : lm_head<false>(d, o, w, lane, S0, W);
    if (lane == 0) s_head_done = S.done;
  }
  // diagonal-block inverses (waves 4 / 5; on waves 6 / 7 after their staging, off the chain waves'
  // SIMDs, they measured no faster)
  if (wv == 4 || wv == 5) {
    int* pd = &s_pdone[side];
    const int nblk = (side == 0 ? m : nB) / 16;
    for (int p = 0; p < nblk; ++p) {
      while (__hip_atomic_load(pd, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) <= p) __builtin_amdgcn_s_sleep(1);
      TR1(56 + 32 * side + 2 * p);   // dbg[256 + 32 side + 2 p]
      me.linv(16 * p);
      if (lane == 0) __hip_atomic_fetch_add(&s_linv[side], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      TR1(57 + 32 * side + 2 * p);
    }
    TR1(10 + side);
  } else if (wv < 2) {
    me.init_panel(P, zr);
#ifdef LORB_CHOL_PHASES
    unsigned long long* phv = d.dbg + 8 * w;  // wave 0, T phase: [0] wait [1] factor [2] store
    if (wv == 0) { if (lane == 0) { phv[0] = phv[1] = phv[2] = 0; } const_cast<BandSide&>(me).phases = phv; }
#endif
    me.chain(P, zr, bad, 0, side == 0 ? m : nB, true, lrd, prd, pwant, pb);
  } else if (wv < 4) {
    me.init_tiles(T);
    me.update(T, 0, side == 0 ? m : nB, lrd, prd, lwant, pb);
  }
  if (wv < 6) C2_STAMP(wv);
  // The T / B back-substitution operators (bsk_block, on the matrix cores), once a side's diagonal
  // inverses are done, on SIMDs 1 and 3 (the M phase's chain and update waves are on 0 and 2): waves
  // 5 / 7 build the top side's (alternate blocks, in the order the back-substitution needs them),
  // waves 1 / 3 the bottom side's after their hand-over to the M phase (below).  The stores drain
  // before the barrier that precedes the back-substitution.
  auto build_ops = [&](int ks, int par) {
    const BandSide& kside = ks == 0 ? top : bot;
    const int nkb = (ks == 0 ? m : nB) / 16;
    wait_ge<true>(&s_linv[ks], nkb);
    TR1(16 + 2 * ks);
    for (int b = nkb - 1 - par; b >= 0; b -= 2) kside.bsk_block(16 * b);
    __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0): the operators are in L2 before the post
    if (lane == 0) __hip_atomic_fetch_add(&s_kdone[ks], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    TR1(17 + 2 * ks);
  };
  if (wv == 5 || wv == 7) build_ops(0, wv == 7);
  // Hand-over to the M phase by flags, not barriers (the diagonal-block inverses of waves 4 / 5
  // may still be running): wave 2 posts that it has read its last L from xt, wave 3 then writes
  // the bottom side's window on M into X = xt (+ xb) and posts it, wave 1 posts zX.
  double* X = xt;  // 48 x 48 in the two exchanges (idle now), original M orientation
  if (wv == 3) {   // the bottom side's window on M, reversed back
    wait_ge<true>(&s_hand[0], 1);
#pragma unroll
    for (int I = 0; I < 3; ++I)
#pragma unroll
      for (int J = 0; J <= I; ++J)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int rho = 16 * I + (lane >> 4) + 4 * r, kap = 16 * J + (lane & 15);
          // unconditional: the upper-triangle slots are never read (no exec-mask branches)
          X[(47 - kap) * 48 + (47 - rho)] = T[tri4(I, J)][r];
          (void)kap; (void)rho;
        }
    if (lane == 0) __hip_atomic_fetch_add(&s_hand[1], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    TR1(2);
  }
  if (wv == 1) {
    if (lane < 48) zX[47 - lane] = zr;
    if (bad) s_bad = 1;
    if (lane == 0) __hip_atomic_fetch_add(&s_hand[2], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  if (wv == 1 || wv == 3) build_ops(1, wv == 3);
  if (wv == 2) {
    TR1(0);
    if (lane == 0) __hip_atomic_fetch_add(&s_hand[0], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    wait_ge<true>(&s_hand[1], 1);
    TR1(1);
  }
  if (wv == 0) wait_ge<true>(&s_hand[2], 1);
  if (wv == 2) {
    // S_M = (S_MM - L_MT L_MT^T) + (S_MM - L_MB L_MB^T) - S_MM ; rows >= m+48 leave the window
#pragma unroll
    for (int I = 0; I < 3; ++I)
#pragma unroll
      for (int J = 0; J <= I; ++J)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int rho = 16 * I + (lane >> 4) + 4 * r, kap = 16 * J + (lane & 15);
          // branch-free: above the diagonal the tiles hold values nobody reads
          T[tri4(I, J)][r] += X[rho * 48 + kap] - top.get(m + rho, m + kap);
        }
#pragma unroll
    for (int J = 0; J < 4; ++J) T[tri4(3, J)] = v4d{0.0, 0.0, 0.0, 0.0};
    TR1(14);
    BandSide topM = top;
    topM.mask = nullptr; topM.pdone = nullptr;
    {  // M's first panel column to the chain wave
      const int ci = lane & 15, ck = lane >> 4;
#pragma unroll
      for (int I = 0; I < 4; ++I)
#pragma unroll
        for (int r = 0; r < 4; ++r) pbt[(16 * I + ck + 4 * r) * 17 + ci] = T[tri4(I, 0)][r];
      if (lane == 0) __hip_atomic_fetch_add(&s_prd[0], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    TR1(15);
    topM.update(T, m, m + 48, &s_lrd[0], &s_prd[0], lwant, pbt);
  } else if (wv == 0) {
    zr = lane < 48 ? zr + zX[lane] - zt[m + lane] : 0.0;
    BandSide topM = top;
    topM.mask = nullptr; topM.pdone = nullptr;
    TR1(3);
    topM.chain(P, zr, bad, m, m + 48, false, &s_lrd[0], &s_prd[0], pwant, pbt);
    TR1(4);
    if (bad) s_bad = 1;
    C2_STAMP(6);
  }
  // (No barrier here.  Wave 0 goes from M's factor straight into the back-substitution,
  // wave 1 waits for y_M by flag, the operators are complete by their builders' flags; a failed
  // factorization (s_bad) only computes values nobody reads and is caught after the last barrier.)
#ifdef LORB_CHOL_PHASES
#define BS_PH(k) do { if (lane == 0) d.dbg[8 * w + (k)] = __builtin_amdgcn_s_memtime(); } while (0)
#else
#define BS_PH(k) do {} while (0)
#endif
  // the side's operator set and window (wave 0 top, wave 1 bottom), then ONE call site
  // of the unrolled T / B back-substitution for both waves (one copy of its code in the
  // instruction cache: the bottom side's copy missed it, 4 k cycles before its first block)
  double cf[16];
  BandSide::BsWin S{0.0};
  if (wv == 0) {
    BS_PH(3);
    wait_ge<true>(&s_kdone[0], 2);
    top.bsk_load(m - 16, cf);  // the first T block's operator, loaded under the M blocks
    S = BandSide::BsWin{top.bs_init(m + 32, 0)};
    TR1(5);
    top.bs_run<false>(S, m + 32, m);                   // y_M (chained triangles)
    BS_PH(4);
    TR1(6);
    if (lane < 48) zb[nB + 47 - lane] = zt[m + lane];  // into the reversed bottom rows
    if (lane == 0) __hip_atomic_fetch_add(&s_hand[0], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  } else if (wv == 1) {
    wait_ge<true>(&s_kdone[1], 2);
    bot.bsk_load(nB - 16, cf);
    // the bottom window's pushes from M's 48 rows: L is final since the B phase, so its 48 entries
    // per lane are loaded before the wait; after it only y_M's broadcast reads and the FMAs remain
    // (four partial sums: a 48-long dependent FMA chain cost ~2 k cycles)
    double lb[48];
    const int brow = bot.bs_row(nB - 16);
#pragma unroll
    for (int k = 0; k < 48; ++k) {
      const bool ok = brow >= 0 && nB + k - brow <= bw;
      const double v = Ab[ok ? bot.idx(nB + k, brow) : bot.base];
      lb[k] = ok ? v : 0.0;
    }
#pragma unroll
    for (int k = 0; k < 48; ++k) asm volatile("" : "+v"(lb[k]));  // loaded here, not sunk past the wait
    wait_ge<true>(&s_hand[0], 2);  // a long wait (the M phase): sleep, do not steal LDS cycles
    BS_PH(6);
    TR1(20);
    double b4[4] = {0.0, 0.0, 0.0, 0.0};
    const double2* zm2 = reinterpret_cast<const double2*>(zb + nB);
#pragma unroll
    for (int k2 = 0; k2 < 24; ++k2) {
      const double2 v = zm2[k2];
      b4[(2 * k2) & 3] = fma(lb[2 * k2], v.x, b4[(2 * k2) & 3]);
      b4[(2 * k2 + 1) & 3] = fma(lb[2 * k2 + 1], v.y, b4[(2 * k2 + 1) & 3]);
    }
    const double bzw = (brow >= 0 ? zb[brow] : 0.0) - ((b4[0] + b4[1]) + (b4[2] + b4[3]));
    S = BandSide::BsWin{bzw};
    TR1(21);
  }
  if (wv < 2) {  // y_T (wave 0) / y_B (wave 1, reversed)
    const BandSide g = wv == 0 ? top : bot;
    g.bs_run_k(S, (wv == 0 ? m : nB) - 16, 0, cf);  // one product per block
    BS_PH(5 + 2 * wv);
    TR1(wv == 0 ? 7 : 12);
  }
#undef BS_PH
  if (wv == 0) C2_STAMP(7);
  __syncthreads();
  TR1(13);
#undef C2_STAMP
#undef TR1
  if (s_bad) {
    if (t == 0) d.st[w].chol_fail = 1;
    return;
  }
  if (HEAD && s_head_done) return;  // the head ended the solve: no candidate
  for (int k = t; k < n; k += NT) d.ycam[W.row_base + k] = k < rt ? zt[k] : zb[n16 - 1 - k];
  for (int ci2 = ep; ep >= 0 && ci2 < W.n_poses; ci2 += 128) {
    const int c = W.pose_base + ci2;
    double xn[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      const int row = 6 * ci2 + k;
      const double y = row < rt ? zt[row] : zb[n16 - 1 - row];
      const double xp = d.x_pose[cur][6 * c + k];
      const double sp = d.scale_pose[6 * c + k];
      xn[k] = xp + (-y) * sp;
      d.x_pose[cur ^ 1][6 * c + k] = xn[k];
    }
    d.rot_cand[c] = lorb::rot_val(xn);
  }
#ifdef LORB_CHOL_TRACE
  if (t == 0) d.dbg[512 * w + 251] = __builtin_amdgcn_s_memtime();  // raw: epilogue issued (thread 0)
#endif
}
template <bool HEAD>
__global__ __launch_bounds__(kChol2sThreads) void k_ba_chol_2s(BaDev d, LMOpt o) { chol_2s_run<HEAD>(d, o, blockIdx.x); }

// the iteration's record (lorb_lm_iteration; S is the state the step was computed from)
__device__ __forceinline__ void lm_record(const BaDev& d, int w, const WinState& S, int outcome, double mcc,
                                          double ncost, double step_norm) {
  if (S.iter < 1 || S.iter > LORB_LM_TRACE_CAP) return;
  lorb_lm_iteration r;
  r.iteration = S.iter; r.outcome = outcome;
  r.cost = S.cost; r.model_cost_change = mcc; r.new_cost = ncost; r.radius = S.radius; r.step_norm = step_norm;
  d.trace[(size_t)w * LORB_LM_TRACE_CAP + S.iter - 1] = r;
}

// K8 decision (lane 0): step validity, tolerances, accept/reject; returns 1 if accepted
__device__ int lm_decide(BaDev d, const LMOpt& o, int w, WinState S, bool valid, double mccs,
                         double ncost, double sn2) {
  const double model_cost_change = -mccs;
  valid = valid && isfinite(model_cost_change) && isfinite(sn2) && model_cost_change > 0.0;
  if (!valid) {
    lm_record(d, w, S, LORB_LM_STEP_INVALID, model_cost_change, ncost, sqrt(sn2));
    if (++S.n_invalid >= o.max_invalid) {
      S.done = 1; S.term = LORB_TERM_FAILURE;
    } else {
      S.radius = S.radius / S.decrease_factor;
      S.decrease_factor *= 2.0;
      S.last_successful = 0;
      if (S.iter >= o.max_iter) { S.done = 1; S.term = LORB_TERM_NO_CONVERGENCE; }
    }
    d.st[w] = S;
    return 0;
  }
  S.n_invalid = 0;
  const double new_cost = isfinite(ncost) ? ncost : 1.7976931348623157e308;
  const double step_norm = sqrt(sn2);
  if (step_norm <= o.ptol * (S.x_norm + o.ptol)) {
    lm_record(d, w, S, LORB_LM_STEP_PARAM_TOL, model_cost_change, new_cost, step_norm);
    S.done = 1; S.term = LORB_TERM_PARAMETER_TOL; d.st[w] = S; return 0;
  }
  const double cost_change = S.cost - new_cost;
  if (fabs(cost_change) <= o.ftol * S.cost) {
    lm_record(d, w, S, LORB_LM_STEP_FUNC_TOL, model_cost_change, new_cost, step_norm);
    S.done = 1; S.term = LORB_TERM_FUNCTION_TOL; d.st[w] = S; return 0;
  }
  const double rel = cost_change / model_cost_change;
  lm_record(d, w, S, rel > o.min_rel ? LORB_LM_STEP_ACCEPTED : LORB_LM_STEP_REJECTED, model_cost_change, new_cost,
            step_norm);
  if (rel > o.min_rel) {
    S.cur ^= 1;
    S.relin = 1;
    S.cost = new_cost;  // the accepted point's cost (k_ba_lm_begin recomputes it when relinearising)
    S.n_success++;
    const double tt = 2.0 * rel - 1.0;
    S.radius = S.radius / fmax(1.0 / 3.0, 1.0 - tt * tt * tt);
    S.radius = fmin(o.max_radius, S.radius);
    S.decrease_factor = 2.0;
  } else {
    S.last_successful = 0;
    S.radius = S.radius / S.decrease_factor;
    S.decrease_factor *= 2.0;
  }
  // the head of the next iteration would stop here (iteration budget spent): the solve needs no
  // final linearisation, S.cost is the cost at the final point
  if (S.iter >= o.max_iter) { S.done = 1; S.term = LORB_TERM_NO_CONVERGENCE; }
  d.st[w] = S;
  return rel > o.min_rel;
}

// K8: per-window iteration tail: camera candidate, step validity, tolerances, accept/reject, on one
// wavefront (no workgroup barrier: the decision is broadcast with readfirstlane).  (Run instead by
// the last-finishing point group of the back-substitution -- a per-window counter behind agent-scope
// release / acquire fences -- it measured far slower: on the 8-XCD device those fences write back
// and invalidate L2, C4 step 1.076 -> 1.294 ms.)
template <bool SH>
__device__ __forceinline__ void lm_end_run(const BaDev& d, const LMOpt& o, int w, int lane) {
  const WinState* Sp = d.st + w;
  WinState S = *Sp;
  const BaWin W = d.win[w];  // issued with the state, before the done test
  if (S.done) return;
  bool valid = !S.chol_fail;
  double mccs = 0.0, ncost = 0.0, sn2 = 0.0;
  double xc[6] = {0, 0, 0, 0, 0, 0};  // candidate pose of camera pose_base + lane (kept for its jet)
  if (valid) {
    const int cur = S.cur;
    // the first 64 cameras' poses are requested before the group partials (one round trip for both;
    // the partials' loop would otherwise keep them behind it)
    const int c0 = W.pose_base + lane;
    const bool has0 = lane < W.n_poses;
    double x0[6], xn0[6];
    bool act0 = false;
    if (has0) {
      act0 = d.cam_active[c0];
#pragma unroll
      for (int k = 0; k < 6; ++k) { x0[k] = d.x_pose[cur][6 * c0 + k]; xn0[k] = d.x_pose[cur ^ 1][6 * c0 + k]; }
    }
    if (!SH) group_partials<3, 4, 5, false>(d.part, W.pblk_base, W.n_pblk, lane, mccs, ncost, sn2);
    if (has0) {
#pragma unroll
      for (int k = 0; k < 6; ++k) {
        if (act0) sn2 += (x0[k] - xn0[k]) * (x0[k] - xn0[k]);  // (the same order as the loop below)
        xc[k] = xn0[k];
      }
    }
    for (int c = c0 + 64; c < W.pose_base + W.n_poses; c += 64) {
      const bool active = d.cam_active[c];
      for (int k = 0; k < 6; ++k) {
        const double x = d.x_pose[cur][6 * c + k];
        const double xn = d.x_pose[cur ^ 1][6 * c + k];  // written by k_ba_chol
        if (active) sn2 += (x - xn) * (x - xn);
      }
    }
    mccs = wave_sum(mccs); ncost = wave_sum(ncost); sn2 = wave_sum(sn2);
    if (SH) { mccs += d.wstep[3 * w]; ncost += d.wstep[3 * w + 1]; sn2 += d.wstep[3 * w + 2]; }
  }
  // point-block / Cholesky failures are per iteration: cleared here for the next one (k_ba_ls
  // sets them before k_ba_lm_begin runs)
  S.chol_fail = 0;
  if (SH && lane == 0) d.wfail_part[w] = 0.0;
  int acc = 0;
  if (lane == 0) acc = lm_decide(d, o, w, S, valid, mccs, ncost, sn2);
  acc = __builtin_amdgcn_readfirstlane(acc);  // lane 0's decision, wave-uniform
  // accepted: the candidate is the new linearisation point -> its rotation states for k_ba_ls
  // (an accepted step is a valid one, so the first 64 candidates are already in registers)
  if (acc) {
    if (lane < W.n_poses) d.rot_lin[W.pose_base + lane] = lorb::rot_jet(xc);
    for (int c = W.pose_base + lane + 64; c < W.pose_base + W.n_poses; c += 64)
      d.rot_lin[c] = lorb::rot_jet(d.x_pose[S.cur ^ 1] + 6 * c);
  }
}
template <bool SH>
__global__ __launch_bounds__(64) void k_ba_lm_end(BaDev d, LMOpt o) {
  lm_end_run<SH>(d, o, blockIdx.x, threadIdx.x);
}

// ==========================================================================================
// Point-major Schur path ("PM"; the only one since round 6).  Round 4's
// pair-major path materialised 34 doubles per observation and re-read them once per camera block
// pair a point takes part in (k (k + 1) / 2 pairs for a point seen k times).  Here one kernel per point group
// linearises its observations, eliminates its points and forms the group's contributions to the
// reduced camera system on chip, and writes ONE partial per (group, camera block) of its camera
// window; a second kernel sums the partials of each block in a fixed group order (deterministic, no
// FP64 atomics).  Nothing is stored per observation: the back-substitution re-evaluates the
// linearisation (the same expression on the same inputs: the same bits).
//
// Group window: the group's optimised observations see cameras [cmin, cmin + span) (plan order);
// its blocks (a, b) (a >= b, local to cmin) lie in the band a - b <= bwc (the window's camera-level
// half band), stored row by row: slot(a, dd = a - b).  Per local camera a the partial also holds
// the camera terms diag(Jc^T Jc) (6), Jc^T r (6) and Jc^T g (6).  The diagonal blocks carry
// Jc^T (I - Q Jps^T) Jc = U - A, the off-diagonal ones -A: band = sc (sum) sc^T, plus D^2 on the
// diagonal; rhs = (Jc^T r - Jc^T g) sc.
// ==========================================================================================

__host__ __device__ __forceinline__ int pm_slot(int a, int dd, int bwc) {
  return a <= bwc ? a * (a + 1) / 2 + dd : (bwc + 1) * (bwc + 2) / 2 + (a - bwc - 1) * (bwc + 1) + dd;
}
// slots of a window of `span` cameras
__host__ __device__ __forceinline__ int pm_nslots(int span, int bwc) {
  return span <= 0 ? 0 : pm_slot(span - 1, span - 1 < bwc ? span - 1 : bwc, bwc) + 1;
}
__device__ __forceinline__ void pm_slot_inv(int q, int bwc, int& a, int& dd) {
  const int T = (bwc + 1) * (bwc + 2) / 2;
  if (q < T) {
    a = (int)((sqrt(8.0 * q + 1.0) - 1.0) * 0.5);
    while ((a + 1) * (a + 2) / 2 <= q) ++a;
    while (a * (a + 1) / 2 > q) --a;
    dd = q - a * (a + 1) / 2;
  } else {
    const int r = q - T;
    a = bwc + 1 + r / (bwc + 1);
    dd = r - (r / (bwc + 1)) * (bwc + 1);
  }
}

// LORB_LS_SKIPD 1: phase D's point loop skipped (timing diagnostics only: wrong results)
#ifndef LORB_LS_SKIPD
#define LORB_LS_SKIPD 0
#endif
constexpr int kLsThreads = kGB;
constexpr int kLsWaves = kLsThreads / 64;

// three sums (M1: the second a max) over an NW-wave workgroup: per-wave butterfly, then the waves'
// values in wave order (every thread must call it)
template <int NW, bool M1>
__device__ __forceinline__ void block_red3w(double& a, double& b, double& c, double (*red)[NW]) {
  a = wave_sum(a); b = M1 ? wave_max(b) : wave_sum(b); c = wave_sum(c);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) {
    const int w = threadIdx.x >> 6;
    red[0][w] = a; red[1][w] = b; red[2][w] = c;
  }
  __syncthreads();
  a = red[0][0]; b = red[1][0]; c = red[2][0];
#pragma unroll
  for (int k = 1; k < NW; ++k) { a += red[0][k]; b = M1 ? fmax(b, red[1][k]) : b + red[1][k]; c += red[2][k]; }
}

// The linearisation of one observation at the current linearisation point (k_ba_ls and k_ba_bs2
// evaluate the same expression on the same inputs, so both see the same bits).
__device__ __forceinline__ void pm_lin(const BaDev& d, const BaWin& W, int cur, int p, int c, int fx, double2 uv,
                                       double (&r)[2], double (&Jp)[6], double (&Jc)[12]) {
  double X[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) X[k] = d.x_pt[cur][3 * p + k];
  if (c >= 0) {
    double tr[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) tr[k] = d.x_pose[cur][6 * c + 3 + k];
    residual_jac_s(d.rot_lin[c], tr, X, W.fx, W.fy, W.cx, W.cy, uv.x, uv.y, r, Jp, Jc);
  } else {  // a fixed keyframe: its rotation state from k_ba_init (rot_jet of the same pose: the same bits)
    double tr[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) tr[k] = d.fixed_pose[6 * fx + 3 + k];
    residual_jac_s(d.rot_fix[fx], tr, X, W.fx, W.fy, W.cx, W.cy, uv.x, uv.y, r, Jp, Jc);
  }
}

// PM-K1: one point group per workgroup (observation threads t < kGB; kLsThreads threads for the
// block phase).  Phases:
//   A (observation)  residual + Jacobians in registers, Jp^T Jp / Jp^T r terms to LDS;
//   B (point)        E^T E, E^T r in observation order, Jacobi scale (iteration 0), the point-block
//                    prep (prep_point); the group's camera window (min / max camera);
//   C (observation)  Jps, Q = Jps E^-1, g = Q b; every optimised observation moves to its point's
//                    camera-ordered slot (rank among the point's cameras: no table);
//   D (block row)    thread = (slot, row i): sum over the group's points in point order of row i of
//                    Jc_h^T K Jc_l (K = I - Q_h Jps_l^T on the diagonal, -Q_h Jps_l^T off it), plus
//                    the camera terms on the diagonal; written to the group's partial.
// Cost, point gradient max and |x|^2 partials per group (the head reads them when relinearising).
// SUP (ls_run_sup): the group is one of a super-group's; phase D adds its blocks into the
// super-group's partial (its camera window at the super-group's offset) instead of writing its own.
struct LsSup {
  double* gsp;  // the super-group's partial
  int cmin;     // its first camera (plan numbering)
};
template <bool SUP>
__device__ __forceinline__ void ls_group(const BaDev& d, const LMOpt& o, const unsigned bid, const LsSup& su) {
  __shared__ double s_jc[kGB][12];   // B / C: per point Ei (0..5), bs (6..8), sp (9..11); D: Jc per slot
  __shared__ double s_qj[kGB][12];   // A / B: Jp^T Jp (6) | Jp^T r (3) per observation; D: Q | Jps per slot
  __shared__ double s_rg[kGB][4];    // D: r | g per slot
  __shared__ unsigned long long s_mask[2][kGB];  // per point: its cameras, bits a - cmin (two words: spans <= 128)
  __shared__ int s_po[kGB];
  __shared__ int s_mm[2][kLsWaves];
  __shared__ double red3[3][kLsWaves];
#ifdef LORB_LS_STAMPS
  // dbg[8 g + k]: s_memtime at the kernel's entry (k 0) and after phase A (1), B (2), C (3), D (4),
  // the partial sums (5) of group g (thread 0)
#define LS_STAMP(k) do { if (threadIdx.x == 0) d.dbg[8 * bid + (k)] = __builtin_amdgcn_s_memtime(); } while (0)
#else
#define LS_STAMP(k) do {} while (0)
#endif
  LS_STAMP(0);
#ifdef LORB_LS_STAMPS
  // where the group ran: HW_ID (hwreg 4) << 8 | XCC_ID (hwreg 20); when: the 100 MHz real-time
  // counter at the start (<< 20) | the ticks to the end (slot 7, written at LS_STAMP(5))
  const unsigned long long ls_rt0 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0)
    d.dbg[8 * bid + 6] = ((unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 4) << 8) |
                                (__builtin_amdgcn_s_getreg((31 << 11) | 20) & 255);
#endif
  const PBlk g = d.pblk[bid];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const bool has = t < g.no;
  const int of = g.o0 + min(t, max(g.no - 1, 0));
  const int p_ = has ? d.obs_pt[of] : 0, c_ = has ? d.obs_cam[of] : -1;
  const int fx_ = has ? d.obs_fix[of] : 0;
  const double2 uv = has ? d.obs_uv[of] : make_double2(0.0, 0.0);
  int po0 = 0, po1 = 0;
  // the point phase's global inputs (both iterates: cur is not known yet) go out with the group's
  double Xp[2][3] = {{0, 0, 0}, {0, 0, 0}}, spp[3] = {0, 0, 0};
  if (t < g.cnt) {
    const int p = g.p0 + t;
    po0 = d.pt_obs_off[p]; po1 = d.pt_obs_off[p + 1];
#pragma unroll
    for (int k = 0; k < 3; ++k) { Xp[0][k] = d.x_pt[0][3 * p + k]; Xp[1][k] = d.x_pt[1][3 * p + k]; spp[k] = d.scale_pt[3 * p + k]; }
  }
  const WinState& S = d.st[g.win];
  if (S.done) return;
  const BaWin& W = d.win[g.win];
  const int cur = S.cur;
  const double rad = S.radius;
  if (t < kGB) { s_mask[0][t] = 0ull; s_mask[1][t] = 0ull; }
  // A
  double r[2] = {0, 0}, Jp[6] = {0, 0, 0, 0, 0, 0}, Jc[12];
#pragma unroll
  for (int k = 0; k < 12; ++k) Jc[k] = 0.0;
  double cost = 0.0;
  if (has) {
    pm_lin(d, W, cur, p_, c_, fx_, uv, r, Jp, Jc);
    cost = 0.5 * (r[0] * r[0] + r[1] * r[1]);
    double* v = s_qj[t];
    v[0] = Jp[0] * Jp[0] + Jp[3] * Jp[3]; v[1] = Jp[0] * Jp[1] + Jp[3] * Jp[4];
    v[2] = Jp[0] * Jp[2] + Jp[3] * Jp[5]; v[3] = Jp[1] * Jp[1] + Jp[4] * Jp[4];
    v[4] = Jp[1] * Jp[2] + Jp[4] * Jp[5]; v[5] = Jp[2] * Jp[2] + Jp[5] * Jp[5];
    v[6] = Jp[0] * r[0] + Jp[3] * r[1]; v[7] = Jp[1] * r[0] + Jp[4] * r[1];
    v[8] = Jp[2] * r[0] + Jp[5] * r[1];
  }
  {
    int mn = has && c_ >= 0 ? c_ : 0x7fffffff, mx = has && c_ >= 0 ? c_ : -1;
#pragma unroll
    for (int s = 32; s > 0; s >>= 1) { mn = min(mn, __shfl_xor(mn, s, 64)); mx = max(mx, __shfl_xor(mx, s, 64)); }
    if (lane == 0) { s_mm[0][wv] = mn; s_mm[1][wv] = mx; }
  }
  __syncthreads();
  LS_STAMP(1);
  int cmin = s_mm[0][0], cmax = s_mm[1][0];
#pragma unroll
  for (int k = 1; k < kLsWaves; ++k) { cmin = min(cmin, s_mm[0][k]); cmax = max(cmax, s_mm[1][k]); }
  const int span = cmax >= 0 ? cmax - cmin + 1 : 0;
  // B (point t) -- and the observations' camera bits
  double gm = 0.0, xn2 = 0.0;
  if (t < g.cnt) {
    const int p = g.p0 + t;
    double E[6] = {0, 0, 0, 0, 0, 0}, b[3] = {0, 0, 0};
    for (int e = po0 - g.o0; e < po1 - g.o0; ++e) {
      const double* v = s_qj[e];
#pragma unroll
      for (int k = 0; k < 6; ++k) E[k] += v[k];
#pragma unroll
      for (int k = 0; k < 3; ++k) b[k] += v[6 + k];
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) d.etb[3 * p + k] = b[k];
    double sp[3];
    if (S.iter == 0) {
      sp[0] = 1.0 / (1.0 + sqrt(E[0]));
      sp[1] = 1.0 / (1.0 + sqrt(E[3]));
      sp[2] = 1.0 / (1.0 + sqrt(E[5]));
#pragma unroll
      for (int k = 0; k < 3; ++k) d.scale_pt[3 * p + k] = sp[k];
    } else {
#pragma unroll
      for (int k = 0; k < 3; ++k) sp[k] = spp[k];
    }
    if (po1 > po0) {
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const double X = cur ? Xp[1][k] : Xp[0][k];
        gm = fmax(gm, fabs(X - (X + -b[k])));
        xn2 += X * X;
      }
    }
    double Ei[6], bs[3];
    if (!prep_point(E, b, sp, rad, o, Ei, bs)) prep_fail(d, g.win);
#pragma unroll
    for (int k = 0; k < 6; ++k) { d.pinv[6 * p + k] = Ei[k]; s_jc[t][k] = Ei[k]; }
#pragma unroll
    for (int k = 0; k < 3; ++k) { s_jc[t][6 + k] = bs[k]; s_jc[t][9 + k] = sp[k]; }
    s_po[t] = po0 - g.o0;
  }
  const int lp = p_ - g.p0;
  const int a_ = c_ - cmin;
  if (has && c_ >= 0) atomicOr(&s_mask[a_ >> 6][lp], 1ull << (a_ & 63));
  __syncthreads();
  LS_STAMP(2);
  // C: Jps, Q, g (reads the point data), then the camera-ordered slot
  double Q[6], Js[6], g0 = 0.0, g1 = 0.0;
  int slot = -1;
  if (has && c_ >= 0) {
    const double* pt = s_jc[lp];
#pragma unroll
    for (int k = 0; k < 6; ++k) Js[k] = Jp[k] * pt[9 + k % 3];
#pragma unroll
    for (int rr = 0; rr < 2; ++rr)
#pragma unroll
      for (int j = 0; j < 3; ++j)
        Q[3 * rr + j] = Js[3 * rr] * s3(pt, 0, j) + Js[3 * rr + 1] * s3(pt, 1, j) + Js[3 * rr + 2] * s3(pt, 2, j);
    g0 = Q[0] * pt[6] + Q[1] * pt[7] + Q[2] * pt[8];
    g1 = Q[3] * pt[6] + Q[4] * pt[7] + Q[5] * pt[8];
    const unsigned long long m0 = s_mask[0][lp];
    slot = s_po[lp] + (a_ < 64 ? __popcll(m0 & ((1ull << a_) - 1ull))
                               : __popcll(m0) + __popcll(s_mask[1][lp] & ((1ull << (a_ - 64)) - 1ull)));
  }
  __syncthreads();
  if (slot >= 0) {
#pragma unroll
    for (int k = 0; k < 12; ++k) s_jc[slot][k] = Jc[k];
#pragma unroll
    for (int k = 0; k < 6; ++k) { s_qj[slot][k] = Q[k]; s_qj[slot][6 + k] = Js[k]; }
    s_rg[slot][0] = r[0]; s_rg[slot][1] = r[1]; s_rg[slot][2] = g0; s_rg[slot][3] = g1;
  }
  __syncthreads();
  LS_STAMP(3);
  // D
  const int bwc = W.bwc, nsl = pm_nslots(span, bwc);
  double* gp = SUP ? su.gsp : d.gpart + W.part_base + (size_t)(bid - W.sg_base) * W.part_stride;
  const int aoff = SUP ? cmin - su.cmin : 0;  // the group's first camera in the super-group's window
  if (!SUP && t == 0) d.gspan[bid] = make_int2(span > 0 ? cmin - W.pose_base : 0, span);
  // Lane = slot (its whole 6 x 6 block: the point's loads serve 36 outputs), wave = point subset:
  // every lane of a wave walks the same points (k = wave, wave + 4, ...: a uniform loop, so the next
  // point's mask / offset are requested before this point's FMAs), a lane whose two cameras the
  // point does not share sits the point out.  The four waves' blocks are then summed in wave order
  // through LDS (the observation data is dead by then).  More than 64 slots: waves take 64-slot
  // chunks over all points instead (no point split, no cross-wave sum).
  // A group of few slots (a window's newest points: many points, 1 - 4 cameras) would leave most
  // lanes idle through a long point loop: there R = 2^lr lanes share a slot (R nsl <= 64), lane =
  // (slot, point subset), and their sums are combined by a butterfly (fixed order) first.
  const bool split = nsl <= 64;
  int lr = 0;
  if (split) while (lr < 6 && (nsl << (lr + 1)) <= 64) ++lr;
  const int nrounds = split ? 1 : (nsl + 64 * kLsWaves - 1) / (64 * kLsWaves);
  for (int rd = 0; rd < nrounds; ++rd) {
    const int q = split ? lane >> lr : 64 * (kLsWaves * rd + wv) + lane;
    const int rr = split ? lane & ((1 << lr) - 1) : 0;
    const bool act = q < nsl;
    int a = 0, dd = 0;
    if (act) pm_slot_inv(q, bwc, a, dd);
    const int b = a - dd;
    const bool dg = dd == 0;
    double acc[36], ex[18];
#pragma unroll
    for (int k = 0; k < 36; ++k) acc[k] = 0.0;
#pragma unroll
    for (int k = 0; k < 18; ++k) ex[k] = 0.0;
    const int k0 = split ? (wv << lr) + rr : 0, kst = split ? kLsWaves << lr : 1;
    // the point loop, for group windows of <= 64 cameras (one mask word) or up to 128 (two: the
    // lane's two cameras pick their word, a rank in the high word adds the low word's count)
    auto point_loop = [&](auto wide_tag) {
      constexpr bool kWide = decltype(wide_tag)::value;
      const int wa = kWide ? a >> 6 : 0, wb = kWide ? b >> 6 : 0;
      const unsigned long long ba = act ? 1ull << (a & 63) : 0ull, bb = 1ull << (b & 63);
      unsigned long long m = s_mask[0][k0], mh = kWide ? s_mask[1][k0] : 0ull;
      int po = s_po[k0];
      for (int k = k0; k < g.cnt; k += kst) {
        const unsigned long long mc = m, mch = mh;
        const int pc = po;
        if (k + kst < g.cnt) {  // the next point's
          m = s_mask[0][k + kst]; po = s_po[k + kst];
          if (kWide) mh = s_mask[1][k + kst];
        }
        const unsigned long long ma = kWide && wa ? mch : mc, mb = kWide && wb ? mch : mc;
        if ((ma & ba) && (mb & bb)) {
          const int lo = kWide ? __popcll(mc) : 0;
          const int eh = pc + (kWide && wa ? lo : 0) + __popcll(ma & (ba - 1ull));
          const int el = pc + (kWide && wb ? lo : 0) + __popcll(mb & (bb - 1ull));
          const double* Qh = s_qj[eh];
          const double* Jl = s_qj[el] + 6;
          const double* Ch = s_jc[eh];
          const double* Cl = s_jc[el];
          double k00 = -(Qh[0] * Jl[0] + Qh[1] * Jl[1] + Qh[2] * Jl[2]);
          double k01 = -(Qh[0] * Jl[3] + Qh[1] * Jl[4] + Qh[2] * Jl[5]);
          double k10 = -(Qh[3] * Jl[0] + Qh[4] * Jl[1] + Qh[5] * Jl[2]);
          double k11 = -(Qh[3] * Jl[3] + Qh[4] * Jl[4] + Qh[5] * Jl[5]);
          if (dg) { k00 += 1.0; k11 += 1.0; }
          double cl[12], ch[12];
#pragma unroll
          for (int j = 0; j < 12; ++j) { cl[j] = Cl[j]; ch[j] = Ch[j]; }
#pragma unroll
          for (int i = 0; i < 6; ++i) {
            const double z0 = ch[i] * k00 + ch[6 + i] * k10, z1 = ch[i] * k01 + ch[6 + i] * k11;
#pragma unroll
            for (int j = 0; j < 6; ++j) acc[6 * i + j] = fma(z0, cl[j], fma(z1, cl[6 + j], acc[6 * i + j]));
          }
          if (dg) {
            const double* rg = s_rg[eh];
            const double g0r = rg[0], g1r = rg[1], g2r = rg[2], g3r = rg[3];
#pragma unroll
            for (int i = 0; i < 6; ++i) {
              ex[i] = fma(ch[i], ch[i], fma(ch[6 + i], ch[6 + i], ex[i]));
              ex[6 + i] = fma(ch[i], g0r, fma(ch[6 + i], g1r, ex[6 + i]));
              ex[12 + i] = fma(ch[i], g2r, fma(ch[6 + i], g3r, ex[12 + i]));
            }
          }
        }
      }
    };
    if (!LORB_LS_SKIPD && k0 < g.cnt) {
      if (span > 64) point_loop(std::true_type{});
      else point_loop(std::false_type{});
    }
    for (int m = 1; m < (1 << lr); m <<= 1) {  // the slot's R subsets (lr = 0 unless split)
#pragma unroll
      for (int k = 0; k < 36; ++k) acc[k] += __shfl_xor(acc[k], m, 64);
#pragma unroll
      for (int k = 0; k < 18; ++k) ex[k] += __shfl_xor(ex[k], m, 64);
    }
    const bool own = act && rr == 0;  // the slot's lane after the butterfly
    if (split) {
      // ((w0 + w1) + w2) + w3 through 64 x 36 + 64 x 18 buffers over the dead observation data
      static_assert(64 * 36 <= kGB * 12 && 64 * 18 <= kGB * 12, "reduction buffers");
      __syncthreads();
#pragma unroll
      for (int w = 0; w < kLsWaves; ++w) {
        if (wv == w && own) {
          double* bl = &s_jc[0][0] + 36 * q;
          double* bx = &s_qj[0][0] + 18 * q;
#pragma unroll
          for (int k = 0; k < 36; ++k) { if (w > 0) acc[k] += bl[k]; if (w + 1 < kLsWaves) bl[k] = acc[k]; }
          if (dg) {
#pragma unroll
            for (int k = 0; k < 18; ++k) { if (w > 0) ex[k] += bx[k]; if (w + 1 < kLsWaves) bx[k] = ex[k]; }
          }
        }
        if (w + 1 < kLsWaves) __syncthreads();
      }
    }
    if (own && (!split || wv == kLsWaves - 1)) {
      if (SUP) {  // added in group order into the super-group's partial (zeroed by ls_run_sup)
        double* out = gp + 36 * pm_slot(a + aoff, dd, bwc);
#pragma unroll
        for (int k = 0; k < 36; ++k) out[k] = out[k] + acc[k];
        if (dg) {
          double* gc = gp + W.part_cam + 18 * (a + aoff);
#pragma unroll
          for (int k = 0; k < 18; ++k) gc[k] = gc[k] + ex[k];
        }
      } else {
        double* out = gp + 36 * q;
#pragma unroll
        for (int k = 0; k < 36; ++k) out[k] = acc[k];
        if (dg) {
          double* gc = gp + W.part_cam + 18 * a;
#pragma unroll
          for (int k = 0; k < 18; ++k) gc[k] = ex[k];
        }
      }
    }
  }
  LS_STAMP(4);
  block_red3w<kLsWaves, true>(cost, gm, xn2, red3);
  if (t == 0) { double* P = d.part + 8 * bid; P[0] = cost; P[1] = gm; P[2] = xn2; }
  LS_STAMP(5);
#ifdef LORB_LS_STAMPS
  if (t == 0) d.dbg[8 * bid + 7] = (ls_rt0 << 20) | ((__builtin_amdgcn_s_memrealtime() - ls_rt0) & 0xfffff);
#endif
#undef LS_STAMP
}
__device__ __forceinline__ void ls_run(const BaDev& d, const LMOpt& o, const unsigned bid) {
  if ((int)bid >= d.live[0]) return;
  ls_group<false>(d, o, bid, LsSup{nullptr, 0});
}
__global__ __launch_bounds__(kLsThreads) void k_ba_ls(BaDev d, LMOpt o) { ls_run(d, o, blockIdx.x); }

// Super-group sid: its point groups one after another in one workgroup, their camera-block sums
// added in group order into ONE partial over the union of their camera windows (a window with more
// point groups than two workgroups per CU take in one round: VERDICT r05 item 2, the partials' HBM
// round trip).  The union window comes from the super-group's observations (one pass); its region
// of the partial is zeroed first.
__device__ __forceinline__ void ls_run_sup(const BaDev& d, const LMOpt& o, const unsigned sid) {
  __shared__ int s_r[2][kLsWaves];
  if ((int)sid >= d.live[2]) return;
  const int4 sg = d.sgrp[sid];
  const WinState& S = d.st[sg.x];
  if (S.done) return;
  const BaWin& W = d.win[sg.x];
  const PBlk gf = d.pblk[sg.y], gl = d.pblk[sg.y + sg.z - 1];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  int mn = 0x7fffffff, mx = -1;
  for (int e = gf.o0 + t; e < gl.o0 + gl.no; e += kLsThreads) {
    const int c = d.obs_cam[e];
    if (c >= 0) { mn = min(mn, c); mx = max(mx, c); }
  }
#pragma unroll
  for (int k = 32; k > 0; k >>= 1) { mn = min(mn, __shfl_xor(mn, k, 64)); mx = max(mx, __shfl_xor(mx, k, 64)); }
  if (lane == 0) { s_r[0][wv] = mn; s_r[1][wv] = mx; }
  __syncthreads();
  int cmin = s_r[0][0], cmax = s_r[1][0];
#pragma unroll
  for (int k = 1; k < kLsWaves; ++k) { cmin = min(cmin, s_r[0][k]); cmax = max(cmax, s_r[1][k]); }
  const int span = cmax >= 0 ? cmax - cmin + 1 : 0;
  double* gsp = d.gpart + W.part_base + (size_t)(sid - W.sg_base) * W.part_stride;
  const int nb = 36 * pm_nslots(span, W.bwc), nc = 18 * span;
  for (int i = t; i < nb + nc; i += kLsThreads) gsp[i < nb ? i : W.part_cam + (i - nb)] = 0.0;
  if (t == 0) d.gspan[sid] = make_int2(span > 0 ? cmin - W.pose_base : 0, span);
  __syncthreads();
  for (int k = 0; k < sg.z; ++k) ls_group<true>(d, o, sg.y + k, LsSup{gsp, cmin});
}
__global__ __launch_bounds__(kLsThreads) __attribute__((amdgpu_waves_per_eu(2))) void k_ba_ls_sup(BaDev d, LMOpt o) {
  ls_run_sup(d, o, blockIdx.x);
}

// PM-K2: one workgroup per camera block (h, l) of a window: the partials of the window's groups
// whose camera window holds the block, summed in group order.  Thread = (entry e, subset s); the
// candidate groups of each 256-group chunk are compacted in order, subset s takes every nsub-th.
// MODE 0: the camera terms of the diagonal blocks only (U diag, V: the iteration head's inputs,
//         before k_ba_lm_begin fixes the iteration-0 Jacobi scale);
// MODE 1: the band with D^2 on the diagonal (rank 0) and the rhs (V - R) sc (round 4's pair-major
//         result, for the Cholesky without a head);
// MODE 2: the fused iteration: band without D^2 (k_ba_chol_2s<true> adds it), rhs, U diag and V.
// RT threads per block (256 or 1024: red_threads() picks per plan -- 1024 when a block has many
// candidate groups, or the grid leaves CUs idle; 256 when many blocks share the GPU)
template <int MODE, int RT>
__device__ __forceinline__ void red_run(const BaDev& d, const LMOpt& o, const unsigned bid) {
  constexpr int kRt = RT, kRw = kRt / 64;
  constexpr int kRc = 1024 / kRt;  // groups per thread per chunk: 1024 groups' windows requested at once
  __shared__ int s_cand[kRt * kRc];
  __shared__ int s_a[kRt * kRc];
  __shared__ int s_wc[kRc][kRw];
  __shared__ double s_acc[1024];
  __shared__ double s_tot[54];
  if ((int)bid >= d.live[1]) return;
  const BlockPair bp = d.bp[bid];
  const bool diag = bp.ch == bp.cl;
  if (MODE == 0 && !diag) return;
  const WinState& S = d.st[bp.win];
  const BaWin& W = d.win[bp.win];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  // the finalisation's scales (and MODE 1's camera diagonal) go out with the state
  const int fi = t < 36 ? t / 6 : (t < 42 ? t - 36 : 0), fj = t < 36 ? t % 6 : 0;
  double sci = 1.0, scj = 1.0, udg = 0.0;
  if (MODE != 0) {
    sci = d.scale_pose[6 * bp.ch + fi];
    scj = d.scale_pose[6 * bp.cl + fj];
    if (MODE == 1 && diag) udg = d.U[21 * bp.ch + u21(fi, fi)];
  }
  if (S.done) return;
  const int h = bp.ch - W.pose_base, l = bp.cl - W.pose_base, dd = h - l;
  // entries: [0, 36) the block, [36, 54) the camera terms (U diag, V, R); MODE 0: U diag, V only
  const int e0 = MODE == 0 ? 36 : 0, ne = MODE == 0 ? 12 : (diag ? 54 : 36);
  // The sum's shape does not depend on the width: candidate j of a chunk belongs to subset j mod NS
  // (NS = 1024 / ne, the subsets a 1024-thread block runs one per thread), each subset sums its
  // candidates in order, and the subsets are combined in a fixed tree -- so the 256-, 512- and
  // 1024-thread kernels give the same bits (a window solved alone or batched with others takes the
  // same band).  A narrower block runs up to kSp subsets per thread.
  const int NS = 1024 / ne;
  const int nsub = kRt / ne, e = t % ne, sub = t / ne;
  constexpr int kSp = RT >= 1024 ? 1 : RT >= 512 ? 3 : 5;  // ceil(NS / nsub) for ne in {12, 36, 54}
  double acc[kSp];
#pragma unroll
  for (int q = 0; q < kSp; ++q) acc[q] = 0.0;
  const int g0 = W.sg_base, ng = W.n_sg;
  for (int c0 = 0; c0 < ng; c0 += kRt * kRc) {
    int2 gs[kRc];
#pragma unroll
    for (int u = 0; u < kRc; ++u) {
      const int gi = c0 + kRt * u + t;
      gs[u] = gi < ng ? d.gspan[g0 + gi] : make_int2(0, 0);
    }
    unsigned long long bal[kRc];
#pragma unroll
    for (int u = 0; u < kRc; ++u) {
      const bool cand = gs[u].y > 0 && gs[u].x <= l && h < gs[u].x + gs[u].y;
      bal[u] = __ballot(cand);
      if (lane == 0) s_wc[u][wv] = __popcll(bal[u]);
    }
    __syncthreads();
    // candidates in group order: sub-chunk u, then wave, then lane
    int pre = 0, nc = 0;
#pragma unroll
    for (int u = 0; u < kRc; ++u)
#pragma unroll
      for (int k = 0; k < kRw; ++k) nc += s_wc[u][k];
#pragma unroll
    for (int u = 0; u < kRc; ++u) {
      int pu = pre;
#pragma unroll
      for (int k = 0; k < kRw; ++k) pu += k < wv ? s_wc[u][k] : 0;
      if ((bal[u] >> lane) & 1ull) {
        const int j = pu + __popcll(bal[u] & ((1ull << lane) - 1ull));
        s_cand[j] = c0 + kRt * u + t;
        s_a[j] = h - gs[u].x;
      }
#pragma unroll
      for (int k = 0; k < kRw; ++k) pre += s_wc[u][k];
    }
    __syncthreads();
    if (sub < nsub) {
      const int ee = e0 + e;
      auto at = [&](int j) -> const double* {
        const double* gp = d.gpart + W.part_base + (size_t)s_cand[j] * W.part_stride;
        const int a = s_a[j];
        return ee < 36 ? gp + 36 * pm_slot(a, dd, W.bwc) + ee : gp + W.part_cam + 18 * a + (ee - 36);
      };
      // kRu candidates' loads in flight before they are added (in candidate order: the same sum)
      // (a short last batch adds exact zeros for its missing candidates: the same sum)
      // the thread's subsets advance together, kRu candidates each per round (kSp x kRu loads in
      // flight); every subset still adds its candidates in order
      constexpr int kRu = RT >= 1024 ? 8 : RT >= 512 ? 4 : 2;
      for (int b0 = 0;; b0 += kRu) {
        double v[kSp][kRu];
        bool more = false;
#pragma unroll
        for (int q = 0; q < kSp; ++q) {
          const int s0 = sub + q * nsub;
#pragma unroll
          for (int u = 0; u < kRu; ++u) {
            const int j = s0 + (b0 + u) * NS;
            v[q][u] = s0 < NS && j < nc ? *at(j) : 0.0;
          }
          more |= s0 < NS && s0 + (b0 + kRu) * NS < nc;
        }
#pragma unroll
        for (int q = 0; q < kSp; ++q)
#pragma unroll
          for (int u = 0; u < kRu; ++u) acc[q] += v[q][u];
        if (!more) break;
      }
    }
    __syncthreads();
  }
  if (sub < nsub) {
#pragma unroll
    for (int q = 0; q < kSp; ++q) {
      const int s0 = sub + q * nsub;
      if (s0 < NS) s_acc[e + s0 * ne] = acc[q];
    }
  }
  __syncthreads();
  if (t < ne) {  // the subsets' sums: four interleaved partial sums, then their pairs
    double v4[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll 4
    for (int s = 0; s < NS; ++s) v4[s & 3] += s_acc[t + s * ne];
    s_tot[t] = (v4[0] + v4[1]) + (v4[2] + v4[3]);
  }
  __syncthreads();
  const int c = bp.ch;
  if (MODE == 0) {
    if (t < 6) d.U_part[21 * c + u21(t, t)] = s_tot[t];
    else if (t < 12) d.V_part[6 * c + t - 6] = s_tot[t];
    return;
  }
  double* A = d.env_part + W.env_base;
  if (t < 36) {
    const int i = fi, j = fj;
    if (!diag || j <= i) {
      double v = s_tot[t] * sci * scj;
      if (MODE == 1 && diag && i == j && d.rank0) {
        const double u = udg * sci * sci;
        v += fmin(fmax(u, o.min_diag), o.max_diag) / S.radius;
      }
      band(A, W.bw, 6 * h + i, 6 * l + j) = v;
    }
  } else if (diag && t < 42) {
    const int i = fi;
    d.rhs_part[W.row_base + 6 * h + i] = (s_tot[42 + i] - s_tot[48 + i]) * sci;
    if (MODE == 2) { d.U_part[21 * c + u21(i, i)] = s_tot[36 + i]; d.V_part[6 * c + i] = s_tot[42 + i]; }
  }
}
template <int MODE, int RT>
__global__ __launch_bounds__(RT) void k_ba_red(BaDev d, LMOpt o) { red_run<MODE, RT>(d, o, blockIdx.x); }

// PM-K3: point-group back-substitution with the linearisation re-evaluated
// in registers instead of read back: b_p -= sum_e Jps_e^T (Jc_e y_c(e)), the point step and
// candidate, then the model cost change and the candidate cost per observation.
__device__ __forceinline__ void bs2_run(const BaDev& d, const unsigned bid) {
  __shared__ double sh[kGB][3], sst[kGB][3], sxn[kGB][3], ssp[kGB][3];
  __shared__ double red3[3][kGW];
  if ((int)bid >= d.live[0]) return;
  const PBlk g = d.pblk[bid];
  const int t = threadIdx.x;
  const bool has = t < g.no;
  const int of = g.o0 + min(t, max(g.no - 1, 0));
  const int p_ = has ? d.obs_pt[of] : 0, c_ = has ? d.obs_cam[of] : -1;
  const int fx_ = has ? d.obs_fix[of] : 0;
  const double2 uv = has ? d.obs_uv[of] : make_double2(0.0, 0.0);
  double b[3] = {0, 0, 0}, sp[3] = {0, 0, 0}, Xa[3] = {0, 0, 0}, Xb[3] = {0, 0, 0};
  double Ei[6] = {0, 0, 0, 0, 0, 0};
  int po0 = 0, po1 = 0;
  if (t < g.cnt) {
    const int p = g.p0 + t;
    po0 = d.pt_obs_off[p]; po1 = d.pt_obs_off[p + 1];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      sp[k] = d.scale_pt[3 * p + k];
      b[k] = d.etb[3 * p + k] * sp[k];
      Xa[k] = d.x_pt[0][3 * p + k];
      Xb[k] = d.x_pt[1][3 * p + k];
    }
#pragma unroll
    for (int k = 0; k < 6; ++k) Ei[k] = d.pinv[6 * p + k];
  }
  const WinState& S = d.st[g.win];
  if (S.done || S.chol_fail) return;
  const BaWin& W = d.win[g.win];
  const int cur = S.cur;
  if (t < g.cnt) {
#pragma unroll
    for (int k = 0; k < 3; ++k) ssp[t][k] = sp[k];
  }
  // every camera-indexed input (the step y, the Jacobi scale, the candidate pose) goes out with the
  // linearisation's: one dependent round trip after the observation's indices
  double ys[6] = {0, 0, 0, 0, 0, 0}, tc[3] = {0, 0, 0};
  lorb::RotVal Rc{};
  if (has && c_ >= 0) {
    const double* y = d.ycam + W.row_base + 6 * (c_ - W.pose_base);
#pragma unroll
    for (int i = 0; i < 6; ++i) ys[i] = y[i] * d.scale_pose[6 * c_ + i];
    Rc = d.rot_cand[c_];
#pragma unroll
    for (int k = 0; k < 3; ++k) tc[k] = d.x_pose[cur ^ 1][6 * c_ + 3 + k];
  }
  double r[2] = {0, 0}, Jp[6] = {0, 0, 0, 0, 0, 0}, Jc[12];
#pragma unroll
  for (int k = 0; k < 12; ++k) Jc[k] = 0.0;
  if (has) pm_lin(d, W, cur, p_, c_, fx_, uv, r, Jp, Jc);
  const int lp = p_ - g.p0;
  __syncthreads();
  // W^T y = Jps^T (Jcs y): this observation's push into its point's rhs
  double ya0 = 0.0, ya1 = 0.0;
  if (has) {
    if (c_ >= 0) {
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        ya0 += Jc[i] * ys[i];
        ya1 += Jc[6 + i] * ys[i];
      }
#pragma unroll
      for (int j = 0; j < 3; ++j) sh[t][j] = (Jp[j] * ssp[lp][j]) * ya0 + (Jp[3 + j] * ssp[lp][j]) * ya1;
    } else {
      sh[t][0] = sh[t][1] = sh[t][2] = 0.0;
    }
  }
  __syncthreads();
  double sn2 = 0.0;
  if (t < g.cnt) {
    const int p = g.p0 + t;
    for (int e = po0 - g.o0; e < po1 - g.o0; ++e) {
#pragma unroll
      for (int j = 0; j < 3; ++j) b[j] -= sh[e][j];
    }
    double X[3], step[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) X[k] = cur ? Xb[k] : Xa[k];
#pragma unroll
    for (int j = 0; j < 3; ++j)
      step[j] = -(s3(Ei, j, 0) * b[0] + s3(Ei, j, 1) * b[1] + s3(Ei, j, 2) * b[2]);
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const double xn = X[j] + step[j] * sp[j];
      d.x_pt[cur ^ 1][3 * p + j] = xn;
      sxn[t][j] = xn;
      sst[t][j] = step[j] * sp[j];
      if (po1 > po0) sn2 += (X[j] - xn) * (X[j] - xn);
    }
  }
  __syncthreads();
  double mcc = 0.0, ncost = 0.0;
  if (has) {
    const double Xn[3] = {sxn[lp][0], sxn[lp][1], sxn[lp][2]};
    double m0 = 0.0, m1 = 0.0;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      m0 += Jp[j] * sst[lp][j];
      m1 += Jp[3 + j] * sst[lp][j];
    }
    double rn[2];
    if (c_ >= 0) {
      m0 -= ya0;
      m1 -= ya1;
      residual_s(Rc, tc, Xn, W.fx, W.fy, W.cx, W.cy, uv.x, uv.y, rn);
    } else {
      double tr[3];
#pragma unroll
      for (int k = 0; k < 3; ++k) tr[k] = d.fixed_pose[6 * fx_ + 3 + k];
      residual_s(d.rotv_fix[fx_], tr, Xn, W.fx, W.fy, W.cx, W.cy, uv.x, uv.y, rn);
    }
    mcc = m0 * (r[0] + m0 / 2.0) + m1 * (r[1] + m1 / 2.0);
    ncost = 0.5 * (rn[0] * rn[0] + rn[1] * rn[1]);
  }
  block_red3<false>(mcc, ncost, sn2, red3);
  if (t == 0) {
    double* P = d.part + 8 * bid;
    P[3] = mcc; P[4] = ncost; P[5] = sn2;
  }
}
__global__ __launch_bounds__(kGB) void k_ba_bs2(BaDev d) { bs2_run(d, blockIdx.x); }

// ==========================================================================================
// Plan groups (lorb_ba_group_*): the LM solves of up to kGrpMax plans -- the device-built plans of
// several LocalMapping windows -- launched as ONE set of kernels on one stream, the way a plan of
// several windows is.  Each launch deals its workgroups to the member plans by a block prefix
// (GrpGrid); a workgroup runs the one-plan kernel's code on its member's BaDev (kernel arguments),
// so every member's results are bit-identical to its own solve (the block-pair sums do not depend
// on the k_ba_red width, k_ba_red's note).
// ==========================================================================================
constexpr int kGrpMax = 4;
struct BaGrp {
  BaDev d[kGrpMax];
  int n;
};
struct GrpGrid {
  int pre[kGrpMax + 1];  // workgroups of members [0, k); pre[n] = the launch's workgroups
};
struct GrpInit {  // k_ba_init's per-plan arguments
  int W[kGrpMax], ctot[kGrpMax], n_pt[kGrpMax], nf[kGrpMax];
};
// the member running workgroup b, and b's index in that member's own launch (members without
// workgroups in this launch are skipped: the last member whose prefix is <= b)
__device__ __forceinline__ int grp_member(const GrpGrid& G, int n, unsigned b, unsigned& lb) {
  int k = 0;
#pragma unroll
  for (int i = 1; i < kGrpMax; ++i) k += (i < n && (int)b >= G.pre[i]) ? 1 : 0;
  lb = b - (unsigned)G.pre[k];
  return k;
}
__global__ __launch_bounds__(256) void k_ba_init_g(BaGrp g, GrpGrid G, GrpInit a, LMOpt o) {
  unsigned lb;
  const int k = grp_member(G, g.n, blockIdx.x, lb);
  init_run(g.d[k], a.W[k], a.ctot[k], a.n_pt[k], a.nf[k], o, (int)(lb * 256 + threadIdx.x),
           (G.pre[k + 1] - G.pre[k]) * 256);
}
__global__ __launch_bounds__(kLsThreads) void k_ba_ls_g(BaGrp g, GrpGrid G, LMOpt o) {
  unsigned lb;
  const int k = grp_member(G, g.n, blockIdx.x, lb);
  ls_run(g.d[k], o, lb);
}
template <int MODE, int RT>
__global__ __launch_bounds__(RT) void k_ba_red_g(BaGrp g, GrpGrid G, LMOpt o) {
  unsigned lb;
  const int k = grp_member(G, g.n, blockIdx.x, lb);
  red_run<MODE, RT>(g.d[k], o, lb);
}
__global__ __launch_bounds__(64) void k_ba_lm_begin_g(BaGrp g, GrpGrid G, LMOpt o) {
  unsigned lb;
  const int k = grp_member(G, g.n, blockIdx.x, lb);
  lm_begin_run<false>(g.d[k], o, (int)lb);
}
template <bool HEAD>
__global__ __launch_bounds__(kChol2sThreads) void k_ba_chol_2s_g(BaGrp g, GrpGrid G, LMOpt o) {
  unsigned lb;
  const int k = grp_member(G, g.n, blockIdx.x, lb);
  chol_2s_run<HEAD>(g.d[k], o, (int)lb);
}
__global__ __launch_bounds__(kGB) void k_ba_bs2_g(BaGrp g, GrpGrid G) {
  unsigned lb;
  const int k = grp_member(G, g.n, blockIdx.x, lb);
  bs2_run(g.d[k], lb);
}
__global__ __launch_bounds__(64) void k_ba_lm_end_g(BaGrp g, GrpGrid G, LMOpt o) {
  unsigned lb;
  const int k = grp_member(G, g.n, blockIdx.x, lb);
  lm_end_run<false>(g.d[k], o, (int)lb, threadIdx.x);
}

// ------------------------------------------------------------------------------------------
// pose-only LM (BA::ProjectPoseOptimization), one workgroup per frame, whole solve in-kernel.
// kPoW wavefronts per frame (a12 is the per-frame tracking call: a few hundred residuals): threads
// stride the frame's residuals (the first kPoC per thread held in registers for the whole solve);
// the 28 normal-equation sums are one reduce-scatter per wave (wave_sum_all) plus the waves' sums in
// wave order through LDS, the candidate cost a butterfly plus the same; every thread then carries
// the frame's LM state and solves the 6 x 6 system redundantly (identical bits everywhere, so the
// control flow is uniform).  Two barriers per iteration; the LDS exchange is double-buffered.
#ifdef LORB_PO_STAMPS
// diagnostics (tools/po_stamps.py): s_memtime of frame 0's thread 0 at each phase, in order
__device__ unsigned long long g_po_st[64];
#define PO_STAMP(tag) do { if (blockIdx.x == 0 && threadIdx.x == 0 && po_n < 31) { g_po_st[2 * po_n] = __builtin_amdgcn_s_memtime(); g_po_st[2 * po_n + 1] = (tag); ++po_n; } } while (0)
#else
#define PO_STAMP(tag) do {} while (0)
#endif
constexpr int kPoW = 4, kPoThreads = 64 * kPoW;
constexpr int kPoRegRes = 2 * kPoThreads;  // residuals per frame held in registers (kPoC per thread)
// a small batch's residual offsets as a kernel argument: the residual loads need no round trip first
constexpr int kPoArgF = 16;
struct PoOff { int n; int off[kPoArgF + 1]; };
__global__ __launch_bounds__(kPoThreads) void k_ba_pose_only(PoOff aoff, const int32_t* __restrict__ res_off,
                                                             const float* __restrict__ intr,
                                                             const float* __restrict__ pose_init,
                                                             const float* __restrict__ pts3d,
                                                             const float* __restrict__ obs2d, LMOpt o,
                                                             double* __restrict__ pose_out,
                                                             lorb_ba_summary* __restrict__ sums) {
  __shared__ double s_nv[2][kPoW][28];
  __shared__ double s_cv[2][kPoW];
  const int f = blockIdx.x;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
#ifdef LORB_PO_STAMPS
  int po_n = 0;
#endif
  PO_STAMP(0);
  const int r0 = aoff.n ? aoff.off[f] : res_off[f], r1 = aoff.n ? aoff.off[f + 1] : res_off[f + 1];
  const double fx = intr[4 * f], fyv = intr[4 * f + 1], cx = intr[4 * f + 2], cy = intr[4 * f + 3];
  double xs[6], xn[6], sc[6], JtJ[21], Jtr[6];
#pragma unroll
  for (int k = 0; k < 6; ++k) { xs[k] = (double)pose_init[6 * f + k]; xn[k] = xs[k]; sc[k] = 1.0; }
  if (r1 == r0) {
    if (t < 6) pose_out[6 * f + t] = xs[t];
    if (t == 0) { lorb_ba_summary z = {}; sums[f] = z; }
    return;
  }
  double radius = o.init_radius, df = 2.0;
  int iter = 0, n_success = 0, n_invalid = 0, term = LORB_TERM_NO_CONVERGENCE, last_successful = 1;
  double initial_cost = 0.0, cost = 0.0, gmax = 0.0, xnorm = 0.0;
  bool relin = true;
  int buf = 0;
  // the thread's first kPoC residuals (r0 + t + kPoThreads q) stay in registers for the whole solve;
  // a frame with more reads the rest from memory in each pass (same per-thread order)
  constexpr int kPoC = kPoRegRes / kPoThreads;
  double cX[kPoC][3], cuv[kPoC][2];
#pragma unroll
  for (int q = 0; q < kPoC; ++q) {
    const int r = min(r0 + t + kPoThreads * q, r1 - 1);
#pragma unroll
    for (int k = 0; k < 3; ++k) cX[q][k] = pts3d[3 * r + k];
    cuv[q][0] = obs2d[2 * r]; cuv[q][1] = obs2d[2 * r + 1];
  }
  for (;;) {
    if (relin) {
      PO_STAMP(1);
      double v[32];  // 21 JtJ + 6 Jtr + cost (+ wave_sum_all's padding)
#pragma unroll
      for (int k = 0; k < 28; ++k) v[k] = 0.0;
      const lorb::RotJet R = lorb::rot_jet(xs);  // one frame: rotation state hoisted
      auto acc = [&](const double (&X)[3], double u, double w) {
        double rr[2], Jp[6], Jc[12];
        residual_jac_s(R, xs + 3, X, fx, fyv, cx, cy, u, w, rr, Jp, Jc);
        int q = 0;
#pragma unroll
        for (int a = 0; a < 6; ++a) {
          v[21 + a] = fma(Jc[a], rr[0], fma(Jc[6 + a], rr[1], v[21 + a]));
#pragma unroll
          for (int b = a; b < 6; ++b) { v[q] = fma(Jc[a], Jc[b], fma(Jc[6 + a], Jc[6 + b], v[q])); ++q; }
        }
        v[27] += 0.5 * (rr[0] * rr[0] + rr[1] * rr[1]);
      };
#pragma unroll
      for (int q = 0; q < kPoC; ++q)
        if (r0 + t + kPoThreads * q < r1) acc(cX[q], cuv[q][0], cuv[q][1]);
      for (int r = r0 + t + kPoThreads * kPoC; r < r1; r += kPoThreads) {
        const double X[3] = {pts3d[3 * r], pts3d[3 * r + 1], pts3d[3 * r + 2]};
        acc(X, obs2d[2 * r], obs2d[2 * r + 1]);
      }
      PO_STAMP(2);
      wave_sum_all<28>(v);
      PO_STAMP(3);
      if (lane == 0) {
#pragma unroll
        for (int k = 0; k < 28; ++k) s_nv[buf][wv][k] = v[k];
      }
      __syncthreads();
      PO_STAMP(4);
#pragma unroll
      for (int k = 0; k < 28; ++k) {
        double a = s_nv[buf][0][k];
#pragma unroll
        for (int w = 1; w < kPoW; ++w) a += s_nv[buf][w][k];
        v[k] = a;
      }
      buf ^= 1;
#pragma unroll
      for (int k = 0; k < 21; ++k) JtJ[k] = v[k];
#pragma unroll
      for (int k = 0; k < 6; ++k) Jtr[k] = v[21 + k];
      cost = v[27];
      double gm = 0.0, xn2 = 0.0;
#pragma unroll
      for (int k = 0; k < 6; ++k) { gm = fmax(gm, fabs(xs[k] - (xs[k] + -Jtr[k]))); xn2 += xs[k] * xs[k]; }
      gmax = gm;
      xnorm = sqrt(xn2);
      if (iter == 0) {
        initial_cost = cost;
        const int dg[6] = {0, 6, 11, 15, 18, 20};
#pragma unroll
        for (int k = 0; k < 6; ++k) sc[k] = o.jacobi ? 1.0 / (1.0 + sqrt(JtJ[dg[k]])) : 1.0;
      }
      last_successful = 1;
      relin = false;
    }
    if (iter >= o.max_iter) { term = LORB_TERM_NO_CONVERGENCE; break; }
    if (last_successful && gmax <= o.gtol) { term = LORB_TERM_GRADIENT_TOL; break; }
    if (radius <= o.min_radius) { term = LORB_TERM_MIN_RADIUS; break; }
    iter++;
    // (Js^T Js + D^2) y = Js^T r, D^2 = clamp(diag)/radius ; dense 6x6 Cholesky
    double A[36], y[6];
#pragma unroll
    for (int a = 0; a < 6; ++a) {
#pragma unroll
      for (int b = 0; b < 6; ++b) A[6 * a + b] = JtJ[u21(a, b)] * sc[a] * sc[b];
      y[a] = Jtr[a] * sc[a];
    }
#pragma unroll
    for (int a = 0; a < 6; ++a) A[7 * a] += fmin(fmax(A[7 * a], o.min_diag), o.max_diag) / radius;
    // the six pivots' reciprocal square roots once (v_rsq_f64 + two Newton steps, as k_ba_chol:
    // no IEEE sqrt / division on the chain); the column and both triangular solves multiply by them
    bool ok = true;
    double il[6];
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      double dd = A[7 * j];
#pragma unroll
      for (int k = 0; k < j; ++k) dd -= A[6 * j + k] * A[6 * j + k];
      ok = ok && dd > 0.0;
      il[j] = rsqrt_refined(dd);
#pragma unroll
      for (int i = j + 1; i < 6; ++i) {
        double sv = A[6 * i + j];
#pragma unroll
        for (int k = 0; k < j; ++k) sv -= A[6 * i + k] * A[6 * j + k];
        A[6 * i + j] = sv * il[j];
      }
    }
    double mcc = -1.0;
    if (ok) {
#pragma unroll
      for (int i = 0; i < 6; ++i) { double sv = y[i]; for (int k = 0; k < i; ++k) sv -= A[6 * i + k] * y[k]; y[i] = sv * il[i]; }
#pragma unroll
      for (int i = 5; i >= 0; --i) { double sv = y[i]; for (int k = i + 1; k < 6; ++k) sv -= A[6 * k + i] * y[k]; y[i] = sv * il[i]; }
      // model cost change = -(step.Js^T r + 0.5 step^T Js^T Js step), step = -y
      // on the unscaled step z = sc (-y): lin = z . J^T r, quad = z^T (J^T J z) -- six independent
      // row products, then two dot products (short dependent chains)
      double z[6], w[6];
#pragma unroll
      for (int a = 0; a < 6; ++a) z[a] = sc[a] * -y[a];
#pragma unroll
      for (int a = 0; a < 6; ++a) {
        w[a] = 0.0;
#pragma unroll
        for (int b = 0; b < 6; ++b) w[a] = fma(JtJ[u21(a, b)], z[b], w[a]);
      }
      double lin = 0.0, quad = 0.0;
#pragma unroll
      for (int a = 0; a < 6; ++a) { lin = fma(z[a], Jtr[a], lin); quad = fma(z[a], w[a], quad); }
      mcc = -(lin + 0.5 * quad);
#pragma unroll
      for (int a = 0; a < 6; ++a) xn[a] = xs[a] + (-y[a]) * sc[a];
      ok = isfinite(mcc) && mcc > 0.0;
    }
    if (!ok) {
      if (++n_invalid >= o.max_invalid) { term = LORB_TERM_FAILURE; break; }
      radius /= df; df *= 2.0; last_successful = 0;
      continue;
    }
    n_invalid = 0;
    PO_STAMP(5);
    // candidate cost
    double cv = 0.0;
    {
      const lorb::RotVal R = lorb::rot_val(xn);
#pragma unroll
      for (int q = 0; q < kPoC; ++q)
        if (r0 + t + kPoThreads * q < r1) {
          double rr[2];
          residual_s(R, xn + 3, cX[q], fx, fyv, cx, cy, cuv[q][0], cuv[q][1], rr);
          cv += 0.5 * (rr[0] * rr[0] + rr[1] * rr[1]);
        }
      for (int r = r0 + t + kPoThreads * kPoC; r < r1; r += kPoThreads) {
        const double X[3] = {pts3d[3 * r], pts3d[3 * r + 1], pts3d[3 * r + 2]};
        double rr[2];
        residual_s(R, xn + 3, X, fx, fyv, cx, cy, obs2d[2 * r], obs2d[2 * r + 1], rr);
        cv += 0.5 * (rr[0] * rr[0] + rr[1] * rr[1]);
      }
    }
    PO_STAMP(6);
    cv = wave_sum(cv);
    if (lane == 0) s_cv[buf][wv] = cv;
    __syncthreads();
    PO_STAMP(7);
    cv = s_cv[buf][0];
#pragma unroll
    for (int w = 1; w < kPoW; ++w) cv += s_cv[buf][w];
    buf ^= 1;
    const double new_cost = isfinite(cv) ? cv : 1.7976931348623157e308;
    double sn2 = 0.0;
#pragma unroll
    for (int k = 0; k < 6; ++k) sn2 += (xs[k] - xn[k]) * (xs[k] - xn[k]);
    if (sqrt(sn2) <= o.ptol * (xnorm + o.ptol)) { term = LORB_TERM_PARAMETER_TOL; break; }
    const double cc = cost - new_cost;
    if (fabs(cc) <= o.ftol * cost) { term = LORB_TERM_FUNCTION_TOL; break; }
    const double rel = cc / mcc;
    if (rel > o.min_rel) {
#pragma unroll
      for (int k = 0; k < 6; ++k) xs[k] = xn[k];
      relin = true;
      n_success++;
      const double tt = 2.0 * rel - 1.0;
      radius = fmin(o.max_radius, radius / fmax(1.0 / 3.0, 1.0 - tt * tt * tt));
      df = 2.0;
    } else {
      last_successful = 0;
      radius /= df;
      df *= 2.0;
    }
  }
  PO_STAMP(8);
#pragma unroll
  for (int k = 0; k < 6; ++k)
    if (t == k) pose_out[6 * f + k] = xs[k];
  if (t == 0) {
    lorb_ba_summary sm;
    sm.iterations = iter; sm.successful_steps = n_success; sm.termination = term; sm.pad_ = 0;
    sm.initial_cost = initial_cost; sm.final_cost = cost;
    sums[f] = sm;
  }
}

LMOpt to_dev_opt(const lorb_lm_options* o) {
  LMOpt d;
  d.max_iter = o->max_num_iterations; d.max_invalid = o->max_num_consecutive_invalid_steps;
  d.jacobi = o->jacobi_scaling; d.ftol = o->function_tolerance; d.gtol = o->gradient_tolerance;
  d.ptol = o->parameter_tolerance; d.init_radius = o->initial_trust_region_radius;
  d.max_radius = o->max_trust_region_radius; d.min_radius = o->min_trust_region_radius;
  d.min_rel = o->min_relative_decrease; d.min_diag = o->min_lm_diagonal; d.max_diag = o->max_lm_diagonal;
  return d;
}
// field by field (LMOpt has padding after its ints: a memcmp would see whatever those bytes hold)
bool same_opt(const LMOpt& a, const LMOpt& b) {
  return a.max_iter == b.max_iter && a.max_invalid == b.max_invalid && a.jacobi == b.jacobi && a.ftol == b.ftol &&
         a.gtol == b.gtol && a.ptol == b.ptol && a.init_radius == b.init_radius && a.max_radius == b.max_radius &&
         a.min_radius == b.min_radius && a.min_rel == b.min_rel && a.min_diag == b.min_diag && a.max_diag == b.max_diag;
}

}  // namespace

// ------------------------------------------------------------------------------------------
// device plan construction state (lorb_ba_plan_create_dev; see "Device-resident plan construction")
struct lorb_ba_devbuild {
  int K_cap = 0, P_cap = 0, C = 0, F = 0, Wd = 0;
  int* key_out = nullptr; int* val_out = nullptr;  // point-sorted: point, observation slot
  // build scratch, cleared by one memset per build: pt_cnt (P_cap + 1) | hdr (8) | cov (C * C) |
  // cam_cnt (C) | bits (C * Wd u64, camera x point)
  int* scr = nullptr; size_t scr_bytes = 0;
  int* pt_cnt = nullptr;      // P_cap + 1
  int* hdr = nullptr;         // [0] valid obs, [1] max obs per point, [2] error flags, [3] points
  int* cov = nullptr;         // C * C
  int* cam_cnt = nullptr;     // C
  unsigned long long* bits = nullptr;
  int* perm = nullptr;        // C: input camera -> plan camera
  int pblk_cap = 0, bp_cap = 0, part_cap = 0, gspan_cap = 0, sgrp_cap = 0;
  size_t gpart_cap = 0;  // doubles of BaDev::gpart (the point groups' partials)
  std::vector<int> h_hdr, h_cov, h_cam;
  int* pinned = nullptr; size_t pinned_n = 0;
  double* sol_part = nullptr; size_t sol_n = 0;  // this rank's solve block (== the global one unsharded)
  bool dirty = true;  // the build scratch needs a clearing fill (first build, or after a failed one)
  bool sorted_hint = false;  // the caller's slots are sorted by point: try k_db_sorted first
  std::vector<double> h_red;                     // sharded: the build's host all-reduce
  // per-build structure uploaded in one copy: [BaWin | live (2) | perm (C) | gcam (C) | bp (up_bp_cap)]
  unsigned char* up_dev = nullptr; unsigned char* up_host = nullptr; int up_bp_cap = 0;
  const unsigned char* up_host_dev = nullptr;  // up_host as the device reads it (pinned, mapped)
  size_t off_live = 0, off_perm = 0, off_gcam = 0, off_bp = 0, up_bytes = 0;
  int* gcam = nullptr;  // device: observations per input camera over all ranks (camera activity)
  // camera_order is a function of the adjacency pattern alone: a build whose pattern equals the
  // previous one's (a sliding window usually keeps its banded pattern) reuses that order
  std::vector<char> last_adj;
  std::vector<int> h_copy;  // host copy of the build's readback
  std::vector<int> last_map;
  // a build issued (dev_build_issue: phase 1 and the readback queued) and not yet finished
  hipEvent_t rb_ev = nullptr;
  bool rb_pending = false, rb_sorted = false, rb_fuse = false;
};

struct lorb_ba_plan {
  lorb_ctx* ctx = nullptr;
  int W = 0, Ctot = 0, Ptot = 0, K = 0, NF = 0, n_pblk = 0, n_bp = 0, n_pairs = 0;
  int env_total = 0, n_total = 0, max_env = 0, max_bw = 0, max_env_w = 0, min_n16 = 1 << 30;
  int min_bw = 1 << 30;  // narrowest band of a non-empty window (k_ba_chol_2s needs >= 15)
  // LORB_HOST_PHASE=1 (diagnostics): host time of the device builds' host phase (readback landed ->
  // k_db_gather launched), printed at destruction
  double hp_us = 0.0, hp_sec[6] = {};
  int hp_n = 0;
  std::vector<BaWin> hwin;
  std::vector<void*> allocs;
  BaDev dev{};
  WinState* d_state = nullptr;
  // graph of one LM iteration
  hipGraph_t graph = nullptr;
  hipGraphExec_t gexec = nullptr;
  LMOpt graph_opt{};
  bool has_graph = false;
  unsigned gen = 0;  // bumped whenever the plan's buffers move (a lorb_ba_group's graph then re-captures)
  // launch shape of the captured solve: a rebuild that keeps it (device-built plans launch the
  // point-group / block-pair kernels at capacity) replays the graph without a new capture
  struct GraphKey {
    int kind = -1, lds = 0, memset_env = 0, env_total = 0, grid_pblk = 0, grid_bp = 0, pt_launch = 0, x2_n = 0;
    int red_wide = 0, sup = 0, grid_sg = 0;
    bool operator==(const GraphKey& o) const { return memcmp(this, &o, sizeof(GraphKey)) == 0; }
  } gkey;
  int grid_pblk = 0, grid_bp = 0;  // launch grids of the point-group and block-pair kernels
  int grid_sg = 0;                 // k_ba_ls_sup's grid (partial runs)
  bool has_super = false;          // some window's partial runs hold more than one point group
  int pt_launch = 0;               // points k_ba_init copies (Ptot, or the capacity)
  int* live = nullptr;             // device [n_pblk, n_bp] (BaDev::live)
  lorb_comm* comm = nullptr;  // sharded plan (not owned)
  // exchange 2 of a sharded plan: [send, send + n) -> [recv, ...) (host plans: env | rhs | wfail;
  // device-built plans: rhs | wfail | pad | env, the band's size decides n)
  double* x2_send = nullptr;
  double* x2_recv = nullptr;
  // sharded fused iteration: exchanges 1 and 2 as ONE all-reduce over [lin | pad | solve], which are
  // contiguous (U_part -> U, fx_n doubles)
  size_t fx_n = 0;
  size_t x2_off = 0;  // device-built: offset of env after rhs | wfail | pad
  // per window: camera relabelling (input pose index -> plan camera index; RCM order, §8 item 4)
  std::vector<std::vector<int>> cam_map;
  int chol_kind = -1;         // last launched Cholesky: 0 k_ba_chol, 1 k_ba_chol_w, 2 k_ba_chol_2s
  lorb_ba_devbuild* devb = nullptr;  // device-built plan (lorb_ba_plan_create_dev)
  ~lorb_ba_plan() {
    if (hp_n)
      fprintf(stderr, "lorb_ba_plan: host phase %.2f us per device build (%d builds): checks %.2f order %.2f blocks %.2f "
              "buffers %.2f staging %.2f launch %.2f\n", hp_us / hp_n, hp_n, hp_sec[0] / hp_n, hp_sec[1] / hp_n,
              hp_sec[2] / hp_n, hp_sec[3] / hp_n, hp_sec[4] / hp_n, hp_sec[5] / hp_n);
    // LORB_PM_SPANS=1 (diagnostics): the point groups' camera spans of the last linearisation
    if (dev.gspan && n_pblk > 0 && getenv("LORB_PM_SPANS")) {
      std::vector<int2> gs(n_pblk);
      if (hipStreamSynchronize(ctx->stream) == hipSuccess &&
          hipMemcpy(gs.data(), dev.gspan, sizeof(int2) * n_pblk, hipMemcpyDeviceToHost) == hipSuccess) {
        std::vector<int> sp;
        for (const int2& g : gs) if (g.y > 0) sp.push_back(g.y);
        std::sort(sp.begin(), sp.end());
        if (!sp.empty())
          fprintf(stderr, "lorb_ba_plan: %d point groups (%zu live), %d observations; camera span p50 %d p90 %d max %d\n",
                  n_pblk, sp.size(), K, sp[sp.size() / 2], sp[sp.size() * 9 / 10], sp.back());
      }
    }
#ifdef LORB_LS_STAMPS
    // LORB_LS_PRINT=1: the last k_ba_ls launch's phase cycles (medians over the point groups)
    if (dev.dbg && n_pblk > 0 && getenv("LORB_LS_PRINT")) {
      std::vector<unsigned long long> st((size_t)n_pblk * 8);
      if (hipStreamSynchronize(ctx->stream) == hipSuccess &&
          hipMemcpy(st.data(), dev.dbg, sizeof(unsigned long long) * st.size(), hipMemcpyDeviceToHost) == hipSuccess) {
        fprintf(stderr, "lorb_ba_plan: k_ba_ls phase cycles (median, p90):");
        for (int k = 0; k < 5; ++k) {
          std::vector<long long> v;
          for (int g = 0; g < n_pblk; ++g)
            if (st[8 * g]) v.push_back((long long)(st[8 * g + k + 1] - st[8 * g + k]));
          std::sort(v.begin(), v.end());
          if (!v.empty()) fprintf(stderr, " %c %lld %lld", "ABCDE"[k], v[v.size() / 2], v[v.size() * 9 / 10]);
        }
        fprintf(stderr, "\n");
        // per XCC (s_memtime is per XCC): first start -> last end, and groups that shared a CU with
        // an earlier one (same XCC / SE / SH / CU) -- started after it ended (serial) or not (co-resident)
        std::map<unsigned long long, std::vector<int>> by_cu;
        unsigned long long r0 = ~0ull, r1 = 0;
        std::vector<long long> dur;
        for (int g = 0; g < n_pblk; ++g) {
          if (!st[8 * g]) continue;
          const unsigned long long a = st[8 * g + 7] >> 20, b = a + (st[8 * g + 7] & 0xfffff);
          r0 = std::min(r0, a); r1 = std::max(r1, b);
          dur.push_back((long long)(b - a));
          by_cu[st[8 * g + 6] & 0xff00ffull].push_back(g);  // XCC | CU / SH / SE of HW_ID
        }
        std::sort(dur.begin(), dur.end());
        int shared = 0;
        long long pair_max = 0;
        for (auto& c : by_cu) {
          if (c.second.size() < 2) continue;
          ++shared;
          unsigned long long a = ~0ull, b = 0;
          for (int g : c.second) { a = std::min(a, st[8 * g + 7] >> 20); b = std::max(b, (st[8 * g + 7] >> 20) + (st[8 * g + 7] & 0xfffff)); }
          pair_max = std::max(pair_max, (long long)(b - a));
        }
        if (!dur.empty())
          fprintf(stderr, "lorb_ba_plan: k_ba_ls real time (us): first start -> last end %.2f; group p50 %.2f p90 %.2f max %.2f; "
                  "%zu CUs, %d with > 1 group (their span max %.2f)\n", (r1 - r0) * 0.01, dur[dur.size() / 2] * 0.01,
                  dur[dur.size() * 9 / 10] * 0.01, dur.back() * 0.01, by_cu.size(), shared, pair_max * 0.01);
        // the slowest groups: phases, points / observations, camera span
        std::vector<PBlk> pb(n_pblk);
        std::vector<int2> gs(n_pblk);
        if (hipMemcpy(pb.data(), dev.pblk, sizeof(PBlk) * n_pblk, hipMemcpyDeviceToHost) == hipSuccess &&
            hipMemcpy(gs.data(), dev.gspan, sizeof(int2) * n_pblk, hipMemcpyDeviceToHost) == hipSuccess) {
          std::vector<int> ord;
          for (int g = 0; g < n_pblk; ++g) if (st[8 * g]) ord.push_back(g);
          std::sort(ord.begin(), ord.end(), [&](int a, int b) { return (st[8 * a + 7] & 0xfffff) > (st[8 * b + 7] & 0xfffff); });
          for (size_t i = 0; i < ord.size() && i < 6; ++i) {
            const int g = ord[i];
            fprintf(stderr, "  group %d: %.2f us, points %d obs %d span %d, phases", g, (st[8 * g + 7] & 0xfffff) * 0.01,
                    pb[g].cnt, pb[g].no, gs[g].y);
            for (int k = 0; k < 5; ++k) fprintf(stderr, " %lld", (long long)(st[8 * g + k + 1] - st[8 * g + k]));
            fprintf(stderr, "\n");
          }
        }
      }
    }
#endif
    if (devb) {
      if (devb->rb_ev) (void)hipEventDestroy(devb->rb_ev);
      if (devb->pinned) (void)hipHostFree(devb->pinned);
      if (devb->up_host) (void)hipHostFree(devb->up_host);
      delete devb;
    }
    if (gexec) (void)hipGraphExecDestroy(gexec);
    if (graph) (void)hipGraphDestroy(graph);
    for (void* p : allocs) (void)hipFree(p);
  }
};

namespace {

template <typename T>
int dalloc(lorb_ba_plan* P, size_t n, T** out) {
  void* p = nullptr;
  LORB_HIP(P->ctx, hipMalloc(&p, std::max<size_t>(n, 1) * sizeof(T)));
  P->allocs.push_back(p);
  *out = static_cast<T*>(p);
  return LORB_OK;
}
template <typename T>
int dupload(lorb_ba_plan* P, const std::vector<T>& v, T** out) {
  LORB_TRY(dalloc(P, v.size(), out));
  if (!v.empty())
    LORB_HIP(P->ctx, hipMemcpyAsync(*out, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, P->ctx->stream));
  return LORB_OK;
}

// Camera-level half band of S for a labelling (pos[c] = new index of camera c): max over cameras of
// pos(c) - min(pos(n)) over the cameras n it shares a point with (itself included).
int camera_band(int C, const std::vector<char>& adj, const std::vector<int>& pos) {
  int b = 0;
  for (int c = 0; c < C; ++c) {
    int lo = pos[c];
    for (int n = 0; n < C; ++n)
      if (adj[(size_t)c * C + n]) lo = std::min(lo, pos[n]);
    b = std::max(b, pos[c] - lo);
  }
  return b;
}

// Reverse Cuthill-McKee over the window's camera covisibility graph (adj: C x C, symmetric).  The
// reference orders a LocalPoseOptimization window as [current] + GetCovisibleFrames() sorted by
// ascending covisibility weight (src/bundle_adjust.cpp:210-220, src/frame.cpp:754-774), which
// scatters the non-zero blocks of S over the whole matrix; RCM restores a narrow band, so the
// banded Cholesky applies.  Deterministic: BFS from the lowest-degree unvisited camera (lowest
// index on ties), neighbours in (degree, index) order, then reversed.  Returns old -> new; the
// identity when RCM does not narrow the band.
std::vector<int> camera_order(int C, const std::vector<char>& adj) {
  std::vector<int> id(C), deg(C, 0);
  for (int c = 0; c < C; ++c) {
    id[c] = c;
    for (int n = 0; n < C; ++n) deg[c] += (n != c) && adj[(size_t)c * C + n];
  }
  static const bool off = [] { const char* e = getenv("LORB_NO_RCM"); return e && e[0] == '1'; }();
  if (off || C < 3) return id;
  std::vector<int> order;
  std::vector<char> seen(C, 0);
  order.reserve(C);
  while ((int)order.size() < C) {
    int s = -1;
    for (int c = 0; c < C; ++c)
      if (!seen[c] && (s < 0 || deg[c] < deg[s])) s = c;
    size_t head = order.size();
    order.push_back(s);
    seen[s] = 1;
    while (head < order.size()) {
      const int u = order[head++];
      std::vector<int> nb;
      for (int n = 0; n < C; ++n)
        if (n != u && adj[(size_t)u * C + n] && !seen[n]) nb.push_back(n);
      std::sort(nb.begin(), nb.end(), [&](int a, int b) { return deg[a] != deg[b] ? deg[a] < deg[b] : a < b; });
      for (int n : nb) { seen[n] = 1; order.push_back(n); }
    }
  }
  std::reverse(order.begin(), order.end());
  std::vector<int> pos(C);
  for (int i = 0; i < C; ++i) pos[order[i]] = i;
  return camera_band(C, adj, pos) < camera_band(C, adj, id) ? pos : id;
}

// Point groups and their partials.  A group's camera window [cmin, cmin + span) is held by
// k_ba_ls as two 64-bit words per point, so a group spans at most kPmSpan cameras: device-built
// plans (one window of C cameras) take C <= kPmSpan; host-built plans cut a group where the next
// point would widen it past kPmSpan (any C, as long as no single point's cameras lie more than
// kPmSpan apart in the plan's camera order).
constexpr int kPmSpan = 128;
// the partial budget of one plan: a group's partial holds the camera blocks of a
// window of `span_max` cameras; far above every workload here (C4: 5 MB, the shared window: 0.3 GB)
constexpr size_t kPartBudgetBytes = (size_t)16 << 30;
// a window's partial layout: camera half band, the slots of a group window of span_max cameras, the
// camera terms after them; its groups' partials from `total` on (advanced)
void pm_layout(BaWin& bw, int span_max, long long& total) {
  bw.bwc = bw.n > 0 ? std::max(bw.bw - 5, 0) / 6 : 0;
  span_max = std::max(std::min(span_max, bw.n_poses), 0);
  bw.part_cam = 36 * pm_nslots(span_max, bw.bwc);
  bw.part_stride = bw.part_cam + 18 * span_max;
  bw.part_base = total;
  total += (long long)bw.n_sg * bw.part_stride;
}
// Partial runs: F consecutive point groups per k_ba_ls workgroup, one partial per run, when a window
// has more point groups than one round of two workgroups per CU takes (F = 1 otherwise: C3 / C4
// windows, alone or batched -- F depends on the window only, so a window's bits do not depend on its
// plan's other windows).  LORB_SG_F=k forces k (tests).
int sg_factor(int n_pblk) {
  const char* e = getenv("LORB_SG_F");
  if (e && atoi(e) >= 1) return n_pblk > 1 ? atoi(e) : 1;
  return n_pblk > 512 ? (n_pblk + 479) / 480 : 1;
}
int part_budget_check(lorb_ctx* ctx, long long total) {
  if ((size_t)std::max(total, 1ll) * sizeof(double) > kPartBudgetBytes)
    return lorb::set_error(ctx, LORB_E_NOMEM, "point-group partials need %.1f GB (> %.0f GB budget)",
                           (double)total * sizeof(double) / 1e9, (double)kPartBudgetBytes / 1e9);
  return LORB_OK;
}

int build_plan(lorb_ctx* ctx, int nw, const lorb_ba_window* win_in, lorb_ba_plan* P) {
  // camera relabelling per window (RCM), applied to copies of the pose / observation arrays; the
  // covisibility graph of a sharded window is all-reduced so every rank picks the same order
  P->cam_map.assign(nw, {});
  std::vector<lorb_ba_window> wins(win_in, win_in + nw);
  std::vector<std::vector<int>> frame_buf(nw);
  std::vector<std::vector<float>> pose_buf(nw);
  for (int w = 0; w < nw; ++w) {
    const lorb_ba_window& in = win_in[w];
    const int C = std::max(in.n_poses, 0);
    std::vector<char> adj((size_t)C * C, 0);
    {
      std::vector<std::vector<int>> pf(std::max(in.n_points, 0));
      for (int k = 0; k < in.n_obs; ++k) {
        const int p = in.obs_point[k], f = in.obs_frame[k];
        if (p < 0 || p >= in.n_points || f < 0 || f >= C) continue;  // rejected by the main pass
        pf[p].push_back(f);
      }
      for (auto& v : pf)
        for (int a : v)
          for (int b : v) adj[(size_t)a * C + b] = 1;
      if (P->comm && C > 0) {
        std::vector<double> h(adj.begin(), adj.end());
        LORB_TRY(lorb::comm_allreduce_host(P->comm, h.data(), h.size(), LORB_OP_MAX));
        for (size_t i = 0; i < h.size(); ++i) adj[i] = h[i] > 0.0;
      }
    }
    std::vector<int> map = camera_order(C, adj);
    bool ident = true;
    for (int c = 0; c < C; ++c) ident &= map[c] == c;
    P->cam_map[w] = map;
    if (ident) continue;
    frame_buf[w].assign(in.obs_frame, in.obs_frame + std::max(in.n_obs, 0));
    for (int& f : frame_buf[w])
      if (f >= 0 && f < C) f = map[f];
    pose_buf[w].resize(6 * (size_t)C);
    for (int c = 0; c < C; ++c)
      for (int q = 0; q < 6; ++q) pose_buf[w][6 * (size_t)map[c] + q] = in.pose_init[6 * (size_t)c + q];
    wins[w].obs_frame = frame_buf[w].data();
    wins[w].pose_init = pose_buf[w].data();
  }
  const lorb_ba_window* win = wins.data();
  P->ctx = ctx;
  P->W = nw;
  lorb_comm* comm = P->comm;
  // sharded: band structure, camera activity and observation counts are global -- reduce the
  // per-window first-coupled camera (min), per-camera and per-window observation counts (sum)
  std::vector<std::vector<int>> g_fc(nw);
  std::vector<std::vector<int>> g_cam_obs(nw);
  std::vector<int> g_obs(nw, 0);
  if (comm) {
    size_t nfc = 0;
    for (int w = 0; w < nw; ++w) nfc += (size_t)std::max(win[w].n_poses, 0);
    std::vector<double> hmin(nfc), hsum(nfc + nw);
    size_t o = 0;
    for (int w = 0; w < nw; ++w) {
      const lorb_ba_window& in = win[w];
      std::vector<int> fc(std::max(in.n_poses, 0)), cobs(std::max(in.n_poses, 0), 0);
      for (int c = 0; c < in.n_poses; ++c) fc[c] = c;
      std::vector<std::vector<int>> pf(std::max(in.n_points, 0));
      for (int k = 0; k < in.n_obs; ++k) {
        const int p = in.obs_point[k], f = in.obs_frame[k];
        if (p < 0 || p >= in.n_points || f >= in.n_poses || f < -in.n_fixed) continue;  // rejected below
        if (f >= 0) { pf[p].push_back(f); cobs[f]++; }
      }
      for (auto& v : pf)
        for (int a : v)
          for (int b : v) fc[a] = std::min(fc[a], b);
      for (int c = 0; c < in.n_poses; ++c) { hmin[o + c] = fc[c]; hsum[o + c] = cobs[c]; }
      hsum[nfc + w] = in.n_obs;
      o += in.n_poses;
    }
    LORB_TRY(lorb::comm_allreduce_host(comm, hmin.data(), hmin.size(), LORB_OP_MIN));
    LORB_TRY(lorb::comm_allreduce_host(comm, hsum.data(), hsum.size(), LORB_OP_SUM));
    o = 0;
    for (int w = 0; w < nw; ++w) {
      g_fc[w].resize(win[w].n_poses); g_cam_obs[w].resize(win[w].n_poses);
      for (int c = 0; c < win[w].n_poses; ++c) { g_fc[w][c] = (int)hmin[o + c]; g_cam_obs[w][c] = (int)hsum[o + c]; }
      g_obs[w] = (int)hsum[nfc + w];
      o += win[w].n_poses;
    }
  }
  std::vector<int> cam_active;
  std::vector<int> pt_obs_off(1, 0), obs_cam, obs_fix, obs_pt;
  std::vector<double2> obs_uv;
  std::vector<double> fixed, xpose, xpt;
  std::vector<PBlk> pblk;
  std::vector<int2> gcam;   // per point group: first / last optimised camera (plan numbering)
  std::vector<int4> sgrp;   // partial runs
  std::vector<BlockPair> bps;
  int pose_base = 0, point_base = 0, fix_base = 0, env_base = 0, row_base = 0, n_pairs = 0;
  long long part_total = 0;
  for (int w = 0; w < nw; ++w) {
    const lorb_ba_window& in = win[w];
    if (in.n_poses < 0 || in.n_points < 0 || in.n_obs < 0 || in.n_fixed < 0)
      return lorb::set_error(ctx, LORB_E_INVALID, "window %d: negative sizes", w);
    BaWin bw{};
    bw.pose_base = pose_base; bw.n_poses = in.n_poses;
    bw.point_base = point_base; bw.n_points = in.n_points;
    bw.fx = in.fx; bw.fy = in.fy; bw.cx = in.cx; bw.cy = in.cy;
    bw.obs_base = (int)obs_cam.size(); bw.n_obs = in.n_obs;
    bw.n_obs_all = comm ? g_obs[w] : in.n_obs;
    // obs sorted by point (stable)
    std::vector<int> cnt(in.n_points + 1, 0);
    for (int k = 0; k < in.n_obs; ++k) {
      const int p = in.obs_point[k], f = in.obs_frame[k];
      if (p < 0 || p >= in.n_points) return lorb::set_error(ctx, LORB_E_INVALID, "window %d obs %d: bad point %d", w, k, p);
      if (f >= in.n_poses || f < -in.n_fixed) return lorb::set_error(ctx, LORB_E_INVALID, "window %d obs %d: bad frame %d", w, k, f);
      cnt[p + 1]++;
    }
    for (int p = 0; p < in.n_points; ++p) cnt[p + 1] += cnt[p];
    std::vector<int> order(in.n_obs), fill(in.n_points, 0);
    for (int k = 0; k < in.n_obs; ++k) { const int p = in.obs_point[k]; order[cnt[p] + fill[p]++] = k; }
    const int ob0 = (int)obs_cam.size();
    for (int p = 0; p < in.n_points; ++p) pt_obs_off.push_back(ob0 + cnt[p + 1]);
    for (int e = 0; e < in.n_obs; ++e) {
      const int k = order[e], f = in.obs_frame[k];
      obs_cam.push_back(f >= 0 ? pose_base + f : -1);
      obs_pt.push_back(point_base + in.obs_point[k]);
      obs_fix.push_back(f >= 0 ? -1 : fix_base + (-1 - f));
      obs_uv.push_back(make_double2(in.obs_uv[2 * k], in.obs_uv[2 * k + 1]));
    }
    for (int i = 0; i < 6 * in.n_fixed; ++i) fixed.push_back(in.fixed_pose[i]);
    for (int i = 0; i < 6 * in.n_poses; ++i) xpose.push_back(in.pose_init[i]);
    for (int i = 0; i < 3 * in.n_points; ++i) xpt.push_back(in.point_init[i]);
    // camera activity: observed by this rank (sharded: by some rank)
    {
      std::vector<int> n_cam(in.n_poses, 0);
      for (int e = 0; e < in.n_obs; ++e) { const int c = obs_cam[ob0 + e]; if (c >= 0) n_cam[c - pose_base]++; }
      for (int c = 0; c < in.n_poses; ++c) cam_active.push_back(comm ? (g_cam_obs[w][c] > 0) : n_cam[c] > 0);
    }
    // camera blocks (ch, cl), ch >= cl, that some point couples, with their observation-pair counts
    // (every diagonal block exists); the first coupled camera of each row for the band
    std::map<std::pair<int, int>, int> bmap;
    for (int c = 0; c < in.n_poses; ++c) bmap[{c, c}];
    std::vector<int> fc(in.n_poses);
    for (int c = 0; c < in.n_poses; ++c) fc[c] = c;
    for (int p = 0; p < in.n_points; ++p) {
      const int e0 = ob0 + cnt[p], e1 = ob0 + cnt[p + 1];
      for (int a = e0; a < e1; ++a) {
        const int ca = obs_cam[a];
        if (ca < 0) continue;
        for (int b = e0; b < e1; ++b) {
          const int cb = obs_cam[b];
          if (cb < 0 || cb > ca) continue;
          // the reference keys a point's observations by Frame* (include/map_point.h:83): one per
          // camera (k_ba_ls places a point's observations by camera rank)
          if (cb == ca && a != b)
            return lorb::set_error(ctx, LORB_E_INVALID, "window %d: a point observed twice by one camera", w);
          bmap[{ca - pose_base, cb - pose_base}]++;
          fc[ca - pose_base] = std::min(fc[ca - pose_base], cb - pose_base);
        }
      }
    }
    for (auto& kv : bmap) {
      bps.push_back(BlockPair{w, pose_base + kv.first.first, pose_base + kv.first.second, n_pairs, kv.second});
      n_pairs += kv.second;
    }
    // uniform band of S: bw = max_i (i - first_nonzero_col(i)); exact for Cholesky (no fill
    // outside the envelope, and the zero padding never changes a value)
    const int n = 6 * in.n_poses;
    if (comm)
      for (int c = 0; c < in.n_poses; ++c) fc[c] = std::min(fc[c], g_fc[w][c]);
    int bwid = 0;
    for (int c = 0; c < in.n_poses; ++c) bwid = std::max(bwid, 6 * c + 5 - 6 * fc[c]);
    if (n == 0) bwid = 0;
    bw.env_base = env_base; bw.env_size = n * (bwid + 1); bw.n = n; bw.row_base = row_base; bw.bw = bwid;
    P->max_env = std::max(P->max_env, bw.env_size + 2 * n);
    P->max_bw = std::max(P->max_bw, bwid);
    if (n > 0) P->min_bw = std::min(P->min_bw, bwid);
    {
      const int n16 = (n + 15) & ~15;
      // one-sided K6w: band + z + invd + exchange; two-sided K6t: (n16 + 48) band rows, z, invd,
      // two exchanges, zX -- the larger of the two
      P->max_env_w = std::max(P->max_env_w, std::max(std::max(n16 * (bwid + 1) + 2 * n16 + 64 * 18,
                                                                (n16 + 48) * (bwid + 2) + 2 * 64 * 18 + 48),
                                                       chol2s_words(n16, bwid)));
      if (n16 > 0) P->min_n16 = std::min(P->min_n16, n16);
    }
    env_base += bw.env_size; row_base += n;
    // point groups: consecutive points with <= kGB observations (and <= kGB points) in total whose
    // optimised cameras span <= kPmSpan (k_ba_ls's camera masks); the widest group sizes the partials
    bw.pblk_base = (int)pblk.size();
    int span_max = 0;
    for (int p = 0; p < in.n_points;) {
      PBlk g{w, point_base + p, 0, ob0 + cnt[p], 0};
      int gmin = INT32_MAX, gmax = -1;
      while (p < in.n_points && g.cnt < kGB) {
        const int k = cnt[p + 1] - cnt[p];
        int pmin = INT32_MAX, pmax = -1;
        for (int e = ob0 + cnt[p]; e < ob0 + cnt[p + 1]; ++e)
          if (obs_cam[e] >= 0) { pmin = std::min(pmin, obs_cam[e]); pmax = std::max(pmax, obs_cam[e]); }
        if (k > kGB)
          return lorb::set_error(ctx, LORB_E_UNSUPPORTED, "window %d: point %d has %d observations (a point group holds %d)",
                                 w, p, k, kGB);
        if (pmax - pmin >= kPmSpan)
          return lorb::set_error(ctx, LORB_E_UNSUPPORTED, "window %d: point %d is seen by cameras %d apart (at most %d)",
                                 w, p, pmax - pmin, kPmSpan - 1);
        const int nmin = std::min(gmin, pmin), nmax = std::max(gmax, pmax);
        if (g.cnt > 0 && (g.no + k > kGB || (nmax >= 0 && nmax - nmin >= kPmSpan))) break;
        g.cnt++; g.no += k; ++p;
        gmin = nmin; gmax = nmax;
      }
      if (gmax >= 0) span_max = std::max(span_max, gmax - gmin + 1);
      pblk.push_back(g);
      gcam.push_back(make_int2(gmin, gmax));
    }
    bw.n_pblk = (int)pblk.size() - bw.pblk_base;
    {  // partial runs (super-groups) and the widest run's camera window
      const int F = sg_factor(bw.n_pblk);
      bw.sg_base = (int)sgrp.size();
      if (F > 1) span_max = 0;
      for (int g = 0; g < bw.n_pblk; g += F) {
        const int ng = std::min(F, bw.n_pblk - g);
        sgrp.push_back(make_int4(w, bw.pblk_base + g, ng, 0));
        int umin = INT32_MAX, umax = -1;
        for (int k = 0; k < ng; ++k) {
          const int2 c = gcam[bw.pblk_base + g + k];
          if (c.y >= 0) { umin = std::min(umin, c.x); umax = std::max(umax, c.y); }
        }
        if (F > 1 && umax >= 0) span_max = std::max(span_max, umax - umin + 1);
      }
      bw.n_sg = (int)sgrp.size() - bw.sg_base;
      P->has_super = P->has_super || F > 1;
    }
    pm_layout(bw, span_max, part_total);
    P->hwin.push_back(bw);
    pose_base += in.n_poses; point_base += in.n_points; fix_base += in.n_fixed;
  }
  P->Ctot = pose_base; P->Ptot = point_base; P->K = (int)obs_cam.size(); P->NF = fix_base;
  LORB_TRY(part_budget_check(ctx, part_total));
  P->n_pblk = (int)pblk.size(); P->n_bp = (int)bps.size(); P->n_pairs = n_pairs;
  P->env_total = env_base; P->n_total = row_base;
  P->grid_pblk = P->n_pblk; P->grid_bp = P->n_bp; P->pt_launch = P->Ptot;
  P->grid_sg = (int)sgrp.size();
  BaDev& d = P->dev;
  BaWin* dwin; PBlk* dpb; BlockPair* dbp; double2* duv;
  int *a1, *a2, *a3;
  double* dfix;
  LORB_TRY(dupload(P, P->hwin, &dwin)); d.win = dwin;
  LORB_TRY(dupload(P, std::vector<int>{P->n_pblk, P->n_bp, (int)sgrp.size()}, &P->live)); d.live = P->live;
  {
    int4* dsg;
    LORB_TRY(dupload(P, sgrp.empty() ? std::vector<int4>{make_int4(0, 0, 0, 0)} : sgrp, &dsg));
    d.sgrp = dsg;
  }
  LORB_TRY(dupload(P, pblk, &dpb)); d.pblk = dpb;
  int* dopt;
  LORB_TRY(dupload(P, obs_pt, &dopt)); d.obs_pt = dopt;
  LORB_TRY(dupload(P, bps, &dbp)); d.bp = dbp;
  LORB_TRY(dupload(P, pt_obs_off, &a1)); d.pt_obs_off = a1;
  LORB_TRY(dupload(P, obs_cam, &a2)); d.obs_cam = a2;
  LORB_TRY(dupload(P, obs_fix, &a3)); d.obs_fix = a3;
  LORB_TRY(dupload(P, obs_uv, &duv)); d.obs_uv = duv;
  LORB_TRY(dupload(P, fixed, &dfix)); d.fixed_pose = dfix;
  LORB_TRY(dupload(P, xpose, &d.x_init_pose));
  LORB_TRY(dupload(P, xpt, &d.x_init_pt));
  LORB_TRY(dupload(P, xpose, &d.x_pose[0]));
  LORB_TRY(dupload(P, xpose, &d.x_pose[1]));
  LORB_TRY(dupload(P, xpt, &d.x_pt[0]));
  LORB_TRY(dupload(P, xpt, &d.x_pt[1]));
  const size_t C = P->Ctot, Pn = P->Ptot;
  LORB_TRY(dalloc(P, C * 6, &d.scale_pose)); LORB_TRY(dalloc(P, Pn * 3, &d.scale_pt));
  LORB_TRY(dalloc(P, Pn * 3, &d.etb)); LORB_TRY(dalloc(P, Pn * 6, &d.pinv));
  int* dact = nullptr;
  LORB_TRY(dupload(P, cam_active, &dact)); d.cam_active = dact;
  // exchange buffers (see BaDev); unsharded plans alias *_part to the global buffers
  const size_t W8 = (size_t)nw, lin_n = C * 27 + 2 * W8, solve_n = (size_t)P->env_total + P->n_total + W8;
  double *lin, *linp, *mx, *mxp, *sol, *solp, *stp, *stpp;
  // [lin | pad | solve] in one block (the sharded fused iteration all-reduces both at once; solve
  // starts 256-byte aligned)
  const size_t lin_pad = (lin_n + 31) & ~(size_t)31;
  LORB_TRY(dalloc(P, lin_pad + solve_n, &lin)); LORB_TRY(dalloc(P, W8, &mx));
  sol = lin + lin_pad;
  LORB_TRY(dalloc(P, 3 * W8, &stp));
  P->fx_n = lin_pad + solve_n;
  if (comm && comm->nranks > 1) {  // one rank: the partials are the global buffers (in-place collectives)
    LORB_TRY(dalloc(P, lin_pad + solve_n, &linp)); LORB_TRY(dalloc(P, W8, &mxp));
    solp = linp + lin_pad;
    LORB_TRY(dalloc(P, 3 * W8, &stpp));
    LORB_HIP(ctx, hipMemsetAsync(linp, 0, sizeof(double) * (lin_pad + solve_n), ctx->stream));
  } else {
    linp = lin; mxp = mx; solp = sol; stpp = stp;
  }
  d.U = lin; d.V = lin + C * 21; d.wlin = lin + C * 27; d.wmax = mx;
  d.U_part = linp; d.V_part = linp + C * 21; d.wlin_part = linp + C * 27; d.wmax_part = mxp;
  d.env = sol; d.rhs = sol + P->env_total; d.wfail = sol + P->env_total + P->n_total;
  d.env_part = solp; d.rhs_part = solp + P->env_total; d.wfail_part = solp + P->env_total + P->n_total;
  P->x2_send = solp; P->x2_recv = sol;
  d.wstep = stp; d.wstep_part = stpp;
  d.sharded = comm ? 1 : 0;
  d.rank0 = comm ? (comm->rank == 0) : 1;
  LORB_TRY(dalloc(P, (size_t)P->Ctot, &d.rot_lin));
  LORB_TRY(dalloc(P, (size_t)P->Ctot, &d.rot_cand));
  LORB_TRY(dalloc(P, (size_t)std::max(P->NF, 1), &d.rot_fix));
  LORB_TRY(dalloc(P, (size_t)std::max(P->NF, 1), &d.rotv_fix));
  if (P->env_total) LORB_HIP(ctx, hipMemsetAsync(d.env, 0, sizeof(double) * P->env_total, ctx->stream));
  LORB_TRY(dalloc(P, (size_t)P->n_total, &d.ycam)); LORB_TRY(dalloc(P, (size_t)P->n_pblk * 8, &d.part));
#ifdef LORB_CHOL_TRACE
  LORB_TRY(dalloc(P, (size_t)nw * 512, &d.dbg));
#elif defined(LORB_LS_STAMPS)
  LORB_TRY(dalloc(P, (size_t)std::max(P->n_pblk, nw) * 8, &d.dbg));
#else
  LORB_TRY(dalloc(P, (size_t)nw * 8, &d.dbg));
#endif
  LORB_TRY(dalloc(P, ((size_t)P->n_total / 16 + nw + 1) * 1024, &d.kco));
  LORB_TRY(dalloc(P, (size_t)nw, &P->d_state)); d.st = P->d_state;
  LORB_TRY(dalloc(P, (size_t)nw * LORB_LM_TRACE_CAP, &d.trace));
  LORB_TRY(dalloc(P, (size_t)std::max(part_total, 1ll), &d.gpart));
  LORB_TRY(dalloc(P, (size_t)std::max(P->grid_sg, 1), &d.gspan));
  LORB_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return LORB_OK;
}

constexpr int kLdsBudget = 160 * 1024 - 2048;

// Cholesky kernel for the plan's band: 2 k_ba_chol_2s, 1 k_ba_chol_w, 0 k_ba_chol, -1 none
int chol_kind_of(const lorb_ba_plan* P) {
  static const bool force_old = [] { const char* e = getenv("LORB_CHOL"); return e && e[0] == 'o'; }();
  static const bool no_2s = [] { const char* e = getenv("LORB_CHOL"); return e && e[0] == 'w'; }();
  if (!P->Ctot) return -1;
  const bool chol_w = !force_old && P->max_bw <= 48 && sizeof(double) * (size_t)P->max_env_w <= (size_t)kLdsBudget;
  // two-sided: its back-substitution uses the full inverse of each 16 x 16 diagonal block, which
  // the band storage holds only for bw >= 15
  const bool chol_2s = chol_w && !no_2s && P->min_n16 >= 128 && P->min_bw >= 15;
  return chol_2s ? 2 : chol_w ? 1 : 0;
}

// doubles of exchange 2 (reduced camera system, rhs, failure flags)
size_t x2_count(const lorb_ba_plan* P) {
  return P->devb ? P->x2_off + (size_t)P->env_total : (size_t)P->env_total + P->n_total + P->W;
}

// k_ba_red's width: 1024 threads when a block has many candidate groups (a window's groups x the
// cameras a group spans / the window's cameras >= 128: the shared window) or the grid leaves CUs
// idle (<= 256 blocks: C3); 512 up to 1024 blocks (C4's 372: 9.8 -> 7.8 us); 256 when many blocks
// share the GPU (several C4 windows per plan)
int red_threads(const lorb_ba_plan* P) {
  const double W = std::max(P->W, 1), cams = std::max((double)P->Ctot / W, 1.0);
  const double cand = (double)P->n_pblk / W * ((P->max_bw + 1) / 6.0) / cams;
  if (P->grid_bp <= 256 || cand >= 128.0) return 1024;
  return P->grid_bp <= 1024 ? 512 : 256;
}
template <int MODE>
void launch_red(const lorb_ba_plan* P, hipStream_t s, const BaDev& d, const LMOpt& o) {
  const int rt = red_threads(P);
  if (rt == 1024) hipLaunchKernelGGL((k_ba_red<MODE, 1024>), dim3(P->grid_bp), dim3(1024), 0, s, d, o);
  else if (rt == 512) hipLaunchKernelGGL((k_ba_red<MODE, 512>), dim3(P->grid_bp), dim3(512), 0, s, d, o);
  else hipLaunchKernelGGL((k_ba_red<MODE, 256>), dim3(P->grid_bp), dim3(256), 0, s, d, o);
}

// the linearisation: one workgroup per point group, or per partial run (k_ba_ls_sup)
void launch_ls(const lorb_ba_plan* P, hipStream_t s, const BaDev& d, const LMOpt& o) {
  lorb::KernelTimer kt(P->ctx, LORB_K_BA_LINEARIZE);
  if (P->has_super) {
    if (P->grid_sg) hipLaunchKernelGGL(k_ba_ls_sup, dim3(P->grid_sg), dim3(kLsThreads), 0, s, d, o);
  } else if (P->grid_pblk) {
    hipLaunchKernelGGL(k_ba_ls, dim3(P->grid_pblk), dim3(kLsThreads), 0, s, d, o);
  }
}

lorb_ba_plan::GraphKey graph_key(const lorb_ba_plan* P) {
  lorb_ba_plan::GraphKey k;
  k.kind = chol_kind_of(P);
  k.lds = k.kind >= 1 ? P->max_env_w : P->max_env + 1000000 * P->max_bw;
  k.memset_env = sizeof(double) * (size_t)P->max_env > (size_t)kLdsBudget;
  k.env_total = k.memset_env ? P->env_total : 0;
  k.grid_pblk = P->grid_pblk; k.grid_bp = P->grid_bp; k.pt_launch = P->pt_launch;
  k.x2_n = P->comm ? (int)x2_count(P) : 0;  // the captured all-reduce's count
  k.red_wide = red_threads(P);
  k.sup = P->has_super ? 1 : 0;
  k.grid_sg = P->grid_sg;
  return k;
}

// one LM iteration (K1..K8) on the ctx stream
int enqueue_linearize(lorb_ba_plan* P, const LMOpt& o) {
  hipStream_t s = P->ctx->stream;
  const BaDev& d = P->dev;
  // the group partials, then the camera terms of the head
  launch_ls(P, s, d, o);
  if (P->grid_bp) {
    lorb::KernelTimer kt(P->ctx, LORB_K_BA_SCHUR);
    launch_red<0>(P, s, d, o);
  }
  if (P->comm) {  // exchange 1: camera blocks + cost / |x|^2 (sum), gradient max (max)
    hipLaunchKernelGGL(k_ba_win_reduce<0>, dim3(P->W), dim3(64), 0, s, d);
    {
      lorb::KernelTimer kt(P->ctx, LORB_K_ALLREDUCE);
      LORB_TRY(lorb::comm_allreduce(P->comm, d.U_part, d.U, (size_t)P->Ctot * 27 + 2 * P->W, LORB_OP_SUM));
      LORB_TRY(lorb::comm_allreduce(P->comm, d.wmax_part, d.wmax, (size_t)P->W, LORB_OP_MAX));
    }
    hipLaunchKernelGGL(k_ba_lm_begin<true>, dim3(P->W), dim3(64), 0, s, d, o);
  } else {
    hipLaunchKernelGGL(k_ba_lm_begin<false>, dim3(P->W), dim3(64), 0, s, d, o);
  }
  return LORB_OK;
}

// one LM iteration on the ctx stream.  first: k_ba_ls -> k_ba_red<0> (camera terms) -> k_ba_lm_begin
// -> k_ba_red<1> -> Cholesky -> k_ba_bs2 -> k_ba_lm_end.  Later iterations of an unsharded plan on
// the two-sided Cholesky run fused: k_ba_red<2> writes the band, rhs and camera terms at once (the
// Jacobi scale is iteration 0's) and the head runs inside the Cholesky (k_ba_lm_begin's work), so
// k_ba_ls -> k_ba_red<2> -> k_ba_chol_2s<true> -> k_ba_bs2 -> k_ba_lm_end: five launches.
int enqueue_iteration(lorb_ba_plan* P, const LMOpt& o, bool first) {
  lorb_ctx* ctx = P->ctx;
  hipStream_t s = ctx->stream;
  const BaDev& d = P->dev;
  static const bool no_fuse = [] { const char* e = getenv("LORB_NO_FUSE"); return e && e[0] == '1'; }();
  const bool fused = !first && chol_kind_of(P) == 2 && !no_fuse;
  if (fused) {
    launch_ls(P, s, d, o);
  } else {
    LORB_TRY(enqueue_linearize(P, o));
  }
  // The LDS Cholesky never writes env, and k_ba_red rewrites every stored entry of
  // every block each iteration, so the band's structural zeros (set at plan creation) persist; the
  // in-place global variant needs them restored.
  const bool chol_in_lds = sizeof(double) * (size_t)P->max_env <= (size_t)kLdsBudget;
  if (P->env_total && !chol_in_lds && !P->comm) LORB_HIP(ctx, hipMemsetAsync(d.env, 0, sizeof(double) * P->env_total, s));
  if (P->grid_bp) {
    lorb::KernelTimer kt(ctx, LORB_K_BA_SCHUR);
    if (fused) launch_red<2>(P, s, d, o);
    else launch_red<1>(P, s, d, o);
  }
  if (P->comm && fused) {
    // the fused sharded iteration: the point partials of the head, then exchanges 1 and 2 as one
    // sum over the contiguous [U | V | cost, |x|^2 | pad | band | rhs | failure flags] (the band's
    // camera blocks and the rhs carry -a / -r only: the Cholesky adds the global U sc sc^T + D^2 and
    // V sc as it stages them) and the gradient max
    hipLaunchKernelGGL(k_ba_win_reduce<0>, dim3(P->W), dim3(64), 0, s, d);
    lorb::KernelTimer kt(ctx, LORB_K_ALLREDUCE);
    LORB_TRY(lorb::comm_allreduce(P->comm, d.U_part, d.U, P->fx_n, LORB_OP_SUM));
    LORB_TRY(lorb::comm_allreduce(P->comm, d.wmax_part, d.wmax, (size_t)P->W, LORB_OP_MAX));
  } else if (P->comm) {  // exchange 2: reduced camera system, rhs, point-block failure flags
    lorb::KernelTimer kt(ctx, LORB_K_ALLREDUCE);
    LORB_TRY(lorb::comm_allreduce(P->comm, P->x2_send, P->x2_recv, x2_count(P), LORB_OP_SUM));
  }
  const int kind = chol_kind_of(P);
  const bool chol_2s = kind == 2, chol_w = kind == 1 || kind == 2;
  P->chol_kind = kind;
  if (P->Ctot && chol_2s) {
    lorb::KernelTimer kt(ctx, LORB_K_BA_CHOLESKY);
    if (fused)
      hipLaunchKernelGGL(k_ba_chol_2s<true>, dim3(P->W), dim3(kChol2sThreads), sizeof(double) * (size_t)P->max_env_w, s, d, o);
    else
      hipLaunchKernelGGL(k_ba_chol_2s<false>, dim3(P->W), dim3(kChol2sThreads), sizeof(double) * (size_t)P->max_env_w, s, d, o);
  } else if (P->Ctot && chol_w) {
    lorb::KernelTimer kt(ctx, LORB_K_BA_CHOLESKY);
    hipLaunchKernelGGL(k_ba_chol_w, dim3(P->W), dim3(256), sizeof(double) * (size_t)P->max_env_w, s, d);
  } else if (P->Ctot) {
    lorb::KernelTimer kt(ctx, LORB_K_BA_CHOLESKY);
    const size_t lds = sizeof(double) * (size_t)P->max_env;
    const bool in_lds = chol_in_lds;
    const int rows = NB + P->max_bw;  // panel rows held in registers by wave 0
    const int rpl = rows <= 64 ? 1 : rows <= 128 ? 2 : rows <= 256 ? 4 : 8;
#define LORB_CHOL(L, R) hipLaunchKernelGGL((k_ba_chol<L, R>), dim3(P->W), dim3(256), L ? lds : 0, s, d)
    if (in_lds) { if (rpl == 1) LORB_CHOL(true, 1); else if (rpl == 2) LORB_CHOL(true, 2); else if (rpl == 4) LORB_CHOL(true, 4); else LORB_CHOL(true, 8); }
    else { if (rpl == 1) LORB_CHOL(false, 1); else if (rpl == 2) LORB_CHOL(false, 2); else if (rpl == 4) LORB_CHOL(false, 4); else LORB_CHOL(false, 8); }
#undef LORB_CHOL
  }
  if (P->grid_pblk) hipLaunchKernelGGL(k_ba_bs2, dim3(P->grid_pblk), dim3(kGB), 0, s, d);
  if (P->comm) {  // exchange 3: model cost change, candidate cost, point |step|^2
    hipLaunchKernelGGL(k_ba_win_reduce<1>, dim3(P->W), dim3(64), 0, s, d);
    {
      lorb::KernelTimer kt(ctx, LORB_K_ALLREDUCE);
      LORB_TRY(lorb::comm_allreduce(P->comm, d.wstep_part, d.wstep, 3 * (size_t)P->W, LORB_OP_SUM));
    }
    hipLaunchKernelGGL(k_ba_lm_end<true>, dim3(P->W), dim3(64), 0, s, d, o);
  } else {
    hipLaunchKernelGGL(k_ba_lm_end<false>, dim3(P->W), dim3(64), 0, s, d, o);
  }
  LORB_CHECK_LAUNCH(ctx);
  return LORB_OK;
}

// the whole solve: x <- initial values, max_iter LM iterations (k_ba_lm_end closes the solve when
// the budget is spent: no final linearisation)
int enqueue_solve(lorb_ba_plan* P, const LMOpt& o) {
  lorb_ctx* ctx = P->ctx;
  {
    const int n = std::max(std::max(std::max(P->W, P->Ctot), P->NF), std::min(3 * P->pt_launch, 256 * 1024));
    hipLaunchKernelGGL(k_ba_init, dim3(lorb::ceil_div(std::max(n, 1), 256)), dim3(256), 0, ctx->stream, P->dev, P->W,
                       P->Ctot, P->pt_launch, P->NF, o);
  }
  LORB_CHECK_LAUNCH(ctx);
  // no iterations: one linearisation (cost, termination) as the head of a first iteration
  if (o.max_iter <= 0) return enqueue_linearize(P, o);
  for (int it = 0; it < o.max_iter; ++it) LORB_TRY(enqueue_iteration(P, o, it == 0));
  return LORB_OK;
}

int plan_solve(lorb_ba_plan* P, const lorb_lm_options* opt) {
  lorb_ctx* ctx = P->ctx;
  LMOpt o = to_dev_opt(opt);
  // per-kernel events cannot live inside a graph, and neither can a host-transport exchange
  static const bool no_graph = [] { const char* e = getenv("LORB_NO_GRAPH"); return e && e[0] == '1'; }();
  const bool timing = ctx->ktime || no_graph || (P->comm && !P->comm->rccl);
  if (timing) return enqueue_solve(P, o);
  const lorb_ba_plan::GraphKey key = graph_key(P);
  if (!P->has_graph || !(key == P->gkey) || !same_opt(P->graph_opt, o)) {
    if (P->gexec) { (void)hipGraphExecDestroy(P->gexec); P->gexec = nullptr; }
    if (P->graph) { (void)hipGraphDestroy(P->graph); P->graph = nullptr; }
    LORB_HIP(ctx, hipStreamBeginCapture(ctx->stream, hipStreamCaptureModeThreadLocal));
    int rc = enqueue_solve(P, o);
    hipGraph_t g = nullptr;
    hipError_t e = hipStreamEndCapture(ctx->stream, &g);
    if (rc != LORB_OK) return rc;
    if (e != hipSuccess) return lorb::set_error(ctx, LORB_E_DEVICE, "graph capture failed: %s", hipGetErrorString(e));
    P->graph = g;
    LORB_HIP(ctx, hipGraphInstantiate(&P->gexec, P->graph, nullptr, nullptr, 0));
    P->graph_opt = o;
    P->gkey = key;
    P->has_graph = true;
  }
  LORB_HIP(ctx, hipGraphLaunch(P->gexec, ctx->stream));
  return LORB_OK;
}

int plan_read(lorb_ba_plan* P, double* const* pose_out, double* const* point_out,
              lorb_ba_summary* sums) {
  lorb_ctx* ctx = P->ctx;
  std::vector<WinState> st(P->W);
  std::vector<std::vector<double>> hp(P->W);  // poses in plan camera order
  LORB_HIP(ctx, hipMemcpyAsync(st.data(), P->d_state, sizeof(WinState) * P->W, hipMemcpyDeviceToHost, ctx->stream));
  LORB_HIP(ctx, hipStreamSynchronize(ctx->stream));
  for (int w = 0; w < P->W; ++w) {
    const BaWin& bw = P->hwin[w];
    const int cur = st[w].cur;
    if (pose_out && pose_out[w] && bw.n_poses) {
      hp[w].resize(6 * (size_t)bw.n_poses);
      LORB_HIP(ctx, hipMemcpyAsync(hp[w].data(), P->dev.x_pose[cur] + 6 * bw.pose_base, sizeof(double) * 6 * bw.n_poses, hipMemcpyDeviceToHost, ctx->stream));
    }
    if (point_out && point_out[w] && bw.n_points)
      LORB_HIP(ctx, hipMemcpyAsync(point_out[w], P->dev.x_pt[cur] + 3 * bw.point_base, sizeof(double) * 3 * bw.n_points, hipMemcpyDeviceToHost, ctx->stream));
    if (sums) {
      lorb_ba_summary s{};
      s.iterations = st[w].iter; s.successful_steps = st[w].n_success; s.termination = st[w].term;
      s.initial_cost = st[w].initial_cost; s.final_cost = st[w].cost;
      if (bw.n_obs_all == 0) { s.iterations = 0; s.termination = LORB_TERM_FUNCTION_TOL; }
      sums[w] = s;
    }
  }
  LORB_HIP(ctx, hipStreamSynchronize(ctx->stream));
  for (int w = 0; w < P->W; ++w) {  // back to the caller's pose order
    if (hp[w].empty()) continue;
    const std::vector<int>& map = P->cam_map[w];
    for (int c = 0; c < P->hwin[w].n_poses; ++c)
      for (int q = 0; q < 6; ++q)
        pose_out[w][6 * (size_t)c + q] = hp[w][6 * (size_t)(map.empty() ? c : map[c]) + q];
  }
  return LORB_OK;
}

}  // namespace

// A plan group (lorb_ba_group_*): member plans (not owned) on one context, solved by one set of
// launches (k_ba_*_g) captured in one graph.  The graph holds the members' BaDev and launch shapes:
// it is re-captured when a member's buffers moved (lorb_ba_plan::gen), its launch shape changed or
// the options differ.
struct lorb_ba_group {
  lorb_ctx* ctx = nullptr;
  std::vector<lorb_ba_plan*> plans;
  hipGraph_t graph = nullptr;
  hipGraphExec_t gexec = nullptr;
  bool has_graph = false;
  LMOpt graph_opt{};
  std::vector<unsigned> gens;
  std::vector<lorb_ba_plan::GraphKey> keys;
  int n_fused = 0, n_captures = 0;  // solves run as one set of launches; graph captures
  ~lorb_ba_group() {
    if (gexec) (void)hipGraphExecDestroy(gexec);
    if (graph) (void)hipGraphDestroy(graph);
  }
};

namespace {

// a group runs as one set of launches when every member is an unsharded plan on the two-sided
// Cholesky (the fused iteration); otherwise its members are solved one after another, each by its
// own path (the same bits either way)
bool group_fused(const lorb_ba_group* G) {
  static const bool no_fuse = [] { const char* e = getenv("LORB_NO_FUSE"); return e && e[0] == '1'; }();
  if (no_fuse || G->plans.size() > (size_t)kGrpMax) return false;
  for (const lorb_ba_plan* P : G->plans)
    if (P->W == 0 || P->comm || P->has_super || chol_kind_of(P) != 2) return false;
  return true;
}

// block prefix of one launch: f(P) workgroups per member
template <typename F>
GrpGrid grp_grid(const lorb_ba_group* G, F f) {
  GrpGrid g{};
  for (size_t k = 0; k < G->plans.size(); ++k) g.pre[k + 1] = g.pre[k] + f(G->plans[k]);
  for (size_t k = G->plans.size() + 1; k <= (size_t)kGrpMax; ++k) g.pre[k] = g.pre[G->plans.size()];
  return g;
}

template <int MODE>
void launch_red_g(const lorb_ba_group* G, hipStream_t s, const BaGrp& bg, const LMOpt& o) {
  const GrpGrid gg = grp_grid(G, [](const lorb_ba_plan* P) { return P->grid_bp; });
  const int n = (int)G->plans.size(), nb = gg.pre[n];
  if (nb == 0) return;
  // the width rule of red_threads over the whole launch (the sums do not depend on it)
  bool wide = nb <= 256;
  for (const lorb_ba_plan* P : G->plans) wide = wide || (red_threads(P) == 1024 && P->grid_bp > 256);
  const int rt = wide ? 1024 : nb <= 1024 ? 512 : 256;
  if (rt == 1024) hipLaunchKernelGGL((k_ba_red_g<MODE, 1024>), dim3(nb), dim3(1024), 0, s, bg, gg, o);
  else if (rt == 512) hipLaunchKernelGGL((k_ba_red_g<MODE, 512>), dim3(nb), dim3(512), 0, s, bg, gg, o);
  else hipLaunchKernelGGL((k_ba_red_g<MODE, 256>), dim3(nb), dim3(256), 0, s, bg, gg, o);
}

// the group's whole solve on the ctx stream (enqueue_solve / enqueue_iteration of every member at once)
int enqueue_group_solve(lorb_ba_group* G, const LMOpt& o) {
  lorb_ctx* ctx = G->ctx;
  hipStream_t s = ctx->stream;
  const int n = (int)G->plans.size();
  BaGrp bg{};
  bg.n = n;
  for (int k = 0; k < n; ++k) bg.d[k] = G->plans[k]->dev;
  {
    GrpInit a{};
    for (int k = 0; k < n; ++k) {
      const lorb_ba_plan* P = G->plans[k];
      a.W[k] = P->W; a.ctot[k] = P->Ctot; a.n_pt[k] = P->pt_launch; a.nf[k] = P->NF;
    }
    const GrpGrid gg = grp_grid(G, [](const lorb_ba_plan* P) {
      const int m = std::max(std::max(std::max(P->W, P->Ctot), P->NF), std::min(3 * P->pt_launch, 256 * 1024));
      return lorb::ceil_div(std::max(m, 1), 256);
    });
    hipLaunchKernelGGL(k_ba_init_g, dim3(gg.pre[n]), dim3(256), 0, s, bg, gg, a, o);
  }
  const GrpGrid g_pb = grp_grid(G, [](const lorb_ba_plan* P) { return P->grid_pblk; });
  const GrpGrid g_w = grp_grid(G, [](const lorb_ba_plan* P) { return P->W; });
  size_t lds = 0;
  for (const lorb_ba_plan* P : G->plans) lds = std::max(lds, sizeof(double) * (size_t)P->max_env_w);
  auto linearise = [&]() {
    lorb::KernelTimer kt(ctx, LORB_K_BA_LINEARIZE);
    if (g_pb.pre[n]) hipLaunchKernelGGL(k_ba_ls_g, dim3(g_pb.pre[n]), dim3(kLsThreads), 0, s, bg, g_pb, o);
  };
  if (o.max_iter <= 0) {  // one linearisation (cost, termination) as the head of a first iteration
    linearise();
    launch_red_g<0>(G, s, bg, o);
    hipLaunchKernelGGL(k_ba_lm_begin_g, dim3(g_w.pre[n]), dim3(64), 0, s, bg, g_w, o);
    LORB_CHECK_LAUNCH(ctx);
    return LORB_OK;
  }
  for (int it = 0; it < o.max_iter; ++it) {
    const bool first = it == 0;
    linearise();
    if (first) {
      {
        lorb::KernelTimer kt(ctx, LORB_K_BA_SCHUR);
        launch_red_g<0>(G, s, bg, o);
      }
      hipLaunchKernelGGL(k_ba_lm_begin_g, dim3(g_w.pre[n]), dim3(64), 0, s, bg, g_w, o);
    }
    for (const lorb_ba_plan* P : G->plans)  // (the two-sided Cholesky holds its band in LDS: none)
      if (P->env_total && sizeof(double) * (size_t)P->max_env > (size_t)kLdsBudget)
        LORB_HIP(ctx, hipMemsetAsync(P->dev.env, 0, sizeof(double) * P->env_total, s));
    {
      lorb::KernelTimer kt(ctx, LORB_K_BA_SCHUR);
      if (first) launch_red_g<1>(G, s, bg, o);
      else launch_red_g<2>(G, s, bg, o);
    }
    {
      lorb::KernelTimer kt(ctx, LORB_K_BA_CHOLESKY);
      if (first)
        hipLaunchKernelGGL(k_ba_chol_2s_g<false>, dim3(g_w.pre[n]), dim3(kChol2sThreads), lds, s, bg, g_w, o);
      else
        hipLaunchKernelGGL(k_ba_chol_2s_g<true>, dim3(g_w.pre[n]), dim3(kChol2sThreads), lds, s, bg, g_w, o);
    }
    if (g_pb.pre[n]) hipLaunchKernelGGL(k_ba_bs2_g, dim3(g_pb.pre[n]), dim3(kGB), 0, s, bg, g_pb);
    hipLaunchKernelGGL(k_ba_lm_end_g, dim3(g_w.pre[n]), dim3(64), 0, s, bg, g_w, o);
  }
  for (lorb_ba_plan* P : G->plans) P->chol_kind = 2;
  LORB_CHECK_LAUNCH(ctx);
  return LORB_OK;
}

int group_solve(lorb_ba_group* G, const lorb_lm_options* opt) {
  lorb_ctx* ctx = G->ctx;
  if (!group_fused(G)) {
    for (lorb_ba_plan* P : G->plans)
      if (P->W > 0) LORB_TRY(plan_solve(P, opt));
    return LORB_OK;
  }
  const LMOpt o = to_dev_opt(opt);
  static const bool no_graph = [] { const char* e = getenv("LORB_NO_GRAPH"); return e && e[0] == '1'; }();
  if (no_graph || ctx->ktime) {  // per-kernel timing: eager launches (events cannot live in a graph)
    LORB_TRY(enqueue_group_solve(G, o));
    G->n_fused++;
    return LORB_OK;
  }
  bool same = G->has_graph && same_opt(G->graph_opt, o);
  for (size_t k = 0; k < G->plans.size() && same; ++k)
    same = G->gens[k] == G->plans[k]->gen && G->keys[k] == graph_key(G->plans[k]);
  if (!same) {
    if (G->gexec) { (void)hipGraphExecDestroy(G->gexec); G->gexec = nullptr; }
    if (G->graph) { (void)hipGraphDestroy(G->graph); G->graph = nullptr; }
    G->has_graph = false;
    LORB_HIP(ctx, hipStreamBeginCapture(ctx->stream, hipStreamCaptureModeThreadLocal));
    const int rc = enqueue_group_solve(G, o);
    hipGraph_t g = nullptr;
    const hipError_t e = hipStreamEndCapture(ctx->stream, &g);
    if (rc != LORB_OK) { if (g) (void)hipGraphDestroy(g); return rc; }
    if (e != hipSuccess) return lorb::set_error(ctx, LORB_E_DEVICE, "group graph capture failed: %s", hipGetErrorString(e));
    G->graph = g;
    LORB_HIP(ctx, hipGraphInstantiate(&G->gexec, G->graph, nullptr, nullptr, 0));
    G->graph_opt = o;
    G->gens.clear(); G->keys.clear();
    for (const lorb_ba_plan* P : G->plans) { G->gens.push_back(P->gen); G->keys.push_back(graph_key(P)); }
    G->has_graph = true;
    G->n_captures++;
  }
  LORB_HIP(ctx, hipGraphLaunch(G->gexec, ctx->stream));
  G->n_fused++;
  return LORB_OK;
}

}  // namespace

// ==========================================================================================
// Device-resident plan construction: the plan of ONE window built from
// observation arrays that already live in HBM (the LocalMapping step appends the new keyframe's
// matches on the device).  The host keeps only the camera-level decisions: one small readback
// (observation / point counts, per-camera counts and the C x C covisibility counts) per build, then
// the camera order (RCM), the (camera, camera) block list, band and kernel choice.  Everything
// per observation, per point and per pair is built by kernels:
//   k_db_keys    validity of the observation slots, per-point counts, camera x point bitsets
//                (a camera seen twice by one point is the bit already set)
//   k_db_scan1   point offsets (one workgroup: exclusive scan, total, largest count)
//   k_db_scatter counting sort by point: slot order within a point restored by k_db_segsort
//                (stable: the caller's order within a point, as a stable radix sort gives it)
//   k_db_cov     covisibility counts of camera pairs = popcount(bits_a & bits_b), per-camera counts
//   k_db_gather  point-sorted observation records (RCM camera labels), initial values (float ->
//                double, camera relabelling), point groups of <= kGB observations (weights k + 1,
//                fixed-size bins), and the zeros the next build starts from
// ==========================================================================================

namespace {



// Build-time scratch of the device plan (one allocation, cleared by the build before -- k_db_gather):
//   pt_cnt[P_cap + 1] | hdr[8] | cov[C * C] | cam_cnt[C] | bits[C * Wd] (u64 words)
// hdr: [0] valid observations, [1] largest count per point, [2] error flags, [3] points.
__global__ __launch_bounds__(256) void k_db_keys(lorb_ba_window_dev w, int C, int F, int Wd,
                                                 int* __restrict__ pt_cnt, int* __restrict__ hdr,
                                                 unsigned long long* __restrict__ bits) {
  const int k = blockIdx.x * 256 + threadIdx.x;
  const int n_obs_in = *w.d_n_obs, n_pt_in = *w.d_n_points;
  // live counts beyond the capacities are an error (flag 8); clamped, so nothing is touched past
  // the plan's allocations
  const int n_obs = min(n_obs_in, w.max_obs), n_pt = min(n_pt_in, w.max_points);
  if (k == 0) {
    hdr[3] = n_pt;
    if (n_obs_in > w.max_obs || n_pt_in > w.max_points || n_obs_in < 0 || n_pt_in < 0) atomicOr(&hdr[2], 8);
  }
  if (k >= n_obs) return;
  const int q = w.d_obs_point[k], f = w.d_obs_frame[k];
  if (f >= -F && f < C) {
    if (q < 0 || q >= n_pt) {
      atomicOr(&hdr[2], 1);
    } else {
      atomicAdd(&pt_cnt[q], 1);
      if (f >= 0) {
        const unsigned long long m = 1ull << (q & 63);
        if (atomicOr(&bits[(size_t)f * Wd + (q >> 6)], m) & m) atomicOr(&hdr[2], 4);
      }
    }
  } else if (f >= C) {
    atomicOr(&hdr[2], 2);
  }
}

// The build's first phase when the observation slots are already sorted by point (the LocalMapping
// map keeps them so; the drop-in's windows are gathered point by point): no counting sort.  One
// thread per slot i <= n_obs: validity, the camera x point bits (a bit already set: a point seen
// twice by one camera); the point offsets from the run boundaries (slot i is the first slot of the
// points (op[i - 1], op[i]], so points without observations get the next point's, and slot n_obs
// closes the points after the last one); the run length of the point starting at i (its largest
// over points).  A slot out of order or unused (frame < -n_fixed) sets flag 16: the host then runs
// the general phase instead.
// The camera x point bits of a workgroup's slots (consecutive points: a few 64-point words) are
// OR-ed in LDS and flushed with one non-returning atomic per (camera, word); a point seen twice by
// one camera is found by the thread that starts the point's run, among the run's frames (the run
// ends at the next run start of the wave's ballot, or by a scan for the wave's last run).  The
// largest run and the error bits are reduced per workgroup before their one atomic each.
// FUSE (C * C ints fit the LDS): the covisibility counts come from the runs too -- the run's start
// thread adds each camera pair of its point (lower triangle: row = the larger camera; the host
// mirrors it after the readback) and each camera's count into LDS tables, flushed with one atomic
// per non-zero entry -- so k_db_cov does not run; and the workgroup's
// histogram of optimised observations by input camera goes to hist[f * NB + block] (NB = 256-slot
// blocks of the live slots, the blocks k_db_gather<true> places), so the placement needs no
// histogram pass of its own.
constexpr int kDbWords = 4;  // 64-point words per workgroup held in LDS (more: global atomics)
constexpr int kDbFuseLds = 64 * 1024;  // LDS bytes the FUSE tables may take
template <bool FUSE>
__global__ __launch_bounds__(256) void k_db_sorted(lorb_ba_window_dev w, int C, int F, int Wd, int* __restrict__ pt_off,
                                                   int* __restrict__ hdr, unsigned long long* __restrict__ bits,
                                                   int* __restrict__ cov, int* __restrict__ cam_cnt) {
  extern __shared__ unsigned long long s_bits[];  // C * kDbWords; FUSE: then cov C * C | cam C (ints)
  int* s_cov = reinterpret_cast<int*>(s_bits + C * kDbWords);
  int* s_cam = s_cov + C * C;
  __shared__ int s_cnt, s_err;
  const int t = threadIdx.x, lane = t & 63;
  const int i = blockIdx.x * 256 + t;
  const int n_obs_in = *w.d_n_obs, n_pt_in = *w.d_n_points;
  const int n_obs = max(min(n_obs_in, w.max_obs), 0), n_pt = max(min(n_pt_in, w.max_points), 0);
  const int* __restrict__ op = w.d_obs_point;
  const int* __restrict__ of = w.d_obs_frame;
  for (int k = t; k < C * kDbWords; k += 256) s_bits[k] = 0ull;
  if (FUSE)
    for (int k = t; k < C * C + C; k += 256) s_cov[k] = 0;
  if (t == 0) { s_cnt = 0; s_err = 0; }
  const int i0 = blockIdx.x * 256;
  const int w0 = i0 < n_obs ? max(op[i0], 0) >> 6 : 0;  // the workgroup's first word
  int err = 0, cnt = 0;
  if (i == 0) {
    hdr[3] = n_pt;
    hdr[0] = n_obs;
    if (n_obs_in > w.max_obs || n_pt_in > w.max_points || n_obs_in < 0 || n_pt_in < 0) err |= 8;
  }
  const int prev = (i > 0 && i <= n_obs) ? op[i - 1] : -1;
  const int q = i < n_obs ? op[i] : n_pt;
  const int f = i < n_obs ? of[i] : -1;
  const bool bound = i <= n_obs && (i == n_obs || prev != q);  // a run starts (or the slots end) here
  const unsigned long long bal = __ballot(bound);
  __syncthreads();
  if (i < n_obs) {
    if (f < -F) err |= 16;
    else if (f >= C) err |= 2;
    else if (q < 0 || q >= n_pt) err |= 1;
    else if (f >= 0) {
      const unsigned long long m = 1ull << (q & 63);
      const int wl = (q >> 6) - w0;
      if (wl >= 0 && wl < kDbWords) atomicOr(&s_bits[f * kDbWords + wl], m);
      else __hip_atomic_fetch_or(&bits[(size_t)f * Wd + (q >> 6)], m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (i <= n_obs) {
    if (prev > q) err |= 16;
    else if (prev != q) {
      const int p1 = min(q, n_pt);
      for (int p = max(prev + 1, 0); p <= p1; ++p) pt_off[p] = i;
      if (i < n_obs) {
        // run end: the next boundary of this wave, else scanned past the wave
        const unsigned long long above = lane < 63 ? bal & (~0ull << (lane + 1)) : 0ull;
        int e;
        if (above) {
          e = i - lane + __builtin_ctzll(above);
        } else {  // the slots past the wave in batches of 8 (one round trip per batch, not per slot)
          e = i - lane + 64;
          for (bool more = true; more;) {
            bool eq[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) eq[u] = e + u < n_obs && op[e + u] == q;
            int run = 0;
#pragma unroll
            for (int u = 7; u >= 0; --u) run = eq[u] ? run + 1 : 0;  // leading matches
            e += run;
            more = run == 8;
          }
          e = min(max(e, i + 1), n_obs);
        }
        cnt = e - i;
        // duplicate cameras within the run (optimised cameras only, as the bitset flags them)
        constexpr int kR = 16;
        int fr[kR];
#pragma unroll
        for (int k = 0; k < kR; ++k) fr[k] = k < cnt ? of[i + k] : -1 - k;
#pragma unroll
        for (int a = 1; a < kR; ++a)
#pragma unroll
          for (int b = 0; b < a; ++b)
            if (fr[a] >= 0 && fr[a] == fr[b]) err |= 4;
        for (int a = kR; a < cnt; ++a) {  // long runs: the rest against everything before it
          const int fa = of[i + a];
          if (fa < 0) continue;
          for (int b = 0; b < a; ++b)
            if (of[i + b] == fa) err |= 4;
        }
        if (FUSE && q >= 0 && q < n_pt) {  // the point's camera pairs and camera counts
#pragma unroll
          for (int a = 0; a < kR; ++a) {
            if (fr[a] < 0 || fr[a] >= C) continue;
            atomicAdd(&s_cam[fr[a]], 1);
#pragma unroll
            for (int b = 0; b < a; ++b)
              if (fr[b] >= 0 && fr[b] < C && fr[b] != fr[a])
                atomicAdd(&s_cov[max(fr[a], fr[b]) * C + min(fr[a], fr[b])], 1);
          }
          for (int a = kR; a < cnt; ++a) {
            const int fa = of[i + a];
            if (fa < 0 || fa >= C) continue;
            atomicAdd(&s_cam[fa], 1);
            for (int b = 0; b < a; ++b) {
              const int fb = of[i + b];
              if (fb >= 0 && fb < C && fb != fa) atomicAdd(&s_cov[max(fa, fb) * C + min(fa, fb)], 1);
            }
          }
        }
      }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) cnt = max(cnt, __shfl_xor(cnt, o, 64));
  if (lane == 0 && cnt) atomicMax(&s_cnt, cnt);
  if (err) atomicOr(&s_err, err);
  __syncthreads();
  for (int k = t; k < C * kDbWords; k += 256) {
    const unsigned long long v = s_bits[k];
    const int wd = w0 + k % kDbWords;
    if (v && wd < Wd)
      __hip_atomic_fetch_or(&bits[(size_t)(k / kDbWords) * Wd + wd], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (FUSE) {
    for (int k = t; k < C * C + C; k += 256) {
      const int v = s_cov[k];  // (cam_cnt follows cov in LDS and in the scratch)
      if (v) __hip_atomic_fetch_add(k < C * C ? &cov[k] : &cam_cnt[k - C * C], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (t == 0) {
    if (s_cnt > __hip_atomic_load(&hdr[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMax(&hdr[1], s_cnt);
    if (s_err) atomicOr(&hdr[2], s_err);
  }
}

// One workgroup: out[0 .. n) = exclusive prefix sums of in[0 .. n) (n_dev: n = *n_dev + 1, the
// live points and one past them).  hdr (optional): hdr[0] = total, hdr[1] = max(in).
__global__ __launch_bounds__(1024) void k_db_scan1(const int* __restrict__ in, int* __restrict__ out, int n,
                                                   const int* __restrict__ n_dev, int* __restrict__ hdr) {
  __shared__ int wsum[16];
  __shared__ int s_tile[lorb::kScanTileLds];
  if (n_dev) n = min(n, *n_dev + 1);
  int mx = 0;
  const int tot = lorb::wg_excl_scan(in, out, n, s_tile, wsum, &mx);
  if (hdr) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = max(mx, __shfl_xor(mx, o, 64));
    if ((threadIdx.x & 63) == 0 && mx) atomicMax(&hdr[1], mx);
    if (threadIdx.x == 0) hdr[0] = tot;
  }
}

// counting sort by point: slot k goes to the end of its point's free range (the counts run down
// to zero, which leaves pt_cnt cleared); k_db_segsort restores the slot order within a point
__global__ __launch_bounds__(256) void k_db_scatter(lorb_ba_window_dev w, int C, int F,
                                                    const int* __restrict__ pt_off, int* __restrict__ pt_cnt,
                                                    int* __restrict__ val) {
  const int k = blockIdx.x * 256 + threadIdx.x;
  const int n_obs = min(*w.d_n_obs, w.max_obs), n_pt = min(*w.d_n_points, w.max_points);
  if (k >= n_obs) return;
  const int q = w.d_obs_point[k], f = w.d_obs_frame[k];
  if (f < -F || f >= C || q < 0 || q >= n_pt) return;
  val[pt_off[q] + atomicSub(&pt_cnt[q], 1) - 1] = k;
}

// one thread per point: its slots ascending.  Points have a few observations (up to kGB - 1):
// up to 16 sort in registers (odd-even transposition network), longer ones by insertion in place.
__global__ __launch_bounds__(256) void k_db_segsort(lorb_ba_window_dev w, const int* __restrict__ pt_off,
                                                    int* __restrict__ val, int* __restrict__ key) {
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= min(*w.d_n_points, w.max_points)) return;
  const int a0 = pt_off[p], a1 = pt_off[p + 1], m = a1 - a0;
  if (m <= 16) {
    int v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = i < m ? val[a0 + i] : 0x7fffffff;
#pragma unroll
    for (int r = 0; r < 16; ++r)
#pragma unroll
      for (int i = r & 1; i + 1 < 16; i += 2) {
        const int lo = min(v[i], v[i + 1]), hi = max(v[i], v[i + 1]);
        v[i] = lo; v[i + 1] = hi;
      }
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if (i < m) { val[a0 + i] = v[i]; key[a0 + i] = p; }
  } else {
    for (int i = a0 + 1; i < a1; ++i) {
      const int x = val[i];
      int j = i - 1;
      while (j >= a0 && val[j] > x) { val[j + 1] = val[j]; --j; }
      val[j + 1] = x;
    }
    for (int i = a0; i < a1; ++i) key[i] = p;
  }
}

// one wavefront per camera pair (a <= b): covisibility = popcount of the AND of their point bitsets
__global__ __launch_bounds__(256) void k_db_cov(int C, int Wd, const unsigned long long* __restrict__ bits,
                                                int* __restrict__ cov, int* __restrict__ cam_cnt) {
  const int pr = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (pr >= C * (C + 1) / 2) return;
  int a = 0, r = pr;  // pr -> (a, b), a <= b, row a holds C - a pairs
  while (r >= C - a) { r -= C - a; ++a; }
  const int b = a + r;
  const unsigned long long* x = bits + (size_t)a * Wd;
  const unsigned long long* y = bits + (size_t)b * Wd;
  int c = 0;
  for (int i = lane; i < Wd; i += 64) c += __popcll(x[i] & y[i]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if (lane == 0) {
    if (a == b) {
      cam_cnt[a] = c;
      cov[a * C + a] = 0;
    } else {
      cov[a * C + b] = c;
      cov[b * C + a] = c;
    }
  }
}

// The work of a build that only needs the pre-readback results and the upload, in one launch:
//  * point-sorted structure arrays; per 256-observation block (blocks < NB) the plan-camera
//    histogram (camera-major hist[c * NB + block], fixed-camera observations not counted);
//  * initial values (float -> double, camera relabelling) and camera activity (k_db_init);
//  * point groups: group g = points [start(g), start(g + 1)), start(g) = the first point p with
//    off[p] + p >= g S (weights k_p + 1, so a group holds <= kGB observations and points; trailing
//    groups can be empty);
//  * zeros: this rank's band, and the build scratch the next build accumulates into (camera x point
//    bitsets, header max / error words, cov / cam_cnt; pt_cnt is left zero by k_db_scatter), so the
//    next build needs no clearing fill.
struct DbFused {
  int C, F, P, G, S, env_n, bits_n;
  int sorted;        // the slots were sorted by point (k_db_sorted): slot e is sorted position e
  unsigned long long* bits;
  int* hdr;
  int* cov;          // cov | cam_cnt (C * C + C ints): zeroed for the next build's k_db_sorted<true>
  int cov_n;
  // the upload is not copied before the launch -- the workgroups copy it from the mapped pinned
  // staging (src -> dst, words), and read perm / gcam from `cams` (kernel arguments), not from the copy
  const int* up_src;
  int* up_dst;
  int up_words;
  int sgf = 1, nsg = 0;  // partial runs: groups per run, runs
  int4* sgrp = nullptr;
};
struct DbCams {  // kernel arguments: device plans hold <= kPmSpan cameras
  int perm[kPmSpan], gcam[kPmSpan];
};
// Point groups: group g = points [start(g), start(g + 1)), start(g) = the smallest p with
// off[p] + p >= g S (P if none), found by one wavefront, 32-ary: each half-wave probes 32 points spread over its
// range per step (one memory round trip) and keeps the gap where the predicate turns true, so a
// 10 k-point window takes 3 round trips instead of 14 dependent loads.  Lanes 0-31 find the start
// of bound b0, lanes 32-63 that of b1.
__device__ __forceinline__ void group_bounds(const int* __restrict__ off, int P, long long b0, long long b1, int lane,
                                             int& s0, int& s1) {
  const int half = lane >> 5, j = lane & 31;
  const long long bound = half ? b1 : b0;
  int lo = 0, hi = P;  // the answer is in [lo, hi] (hi = P: none below P)
  while (__ballot(hi > lo)) {
    const int n = hi - lo;
    bool pr = false;
    if (n > 0) {
      const int q = lo + (int)(((long long)n * (j + 1)) / 33);  // < hi
      pr = (long long)off[q] + q >= bound;
    }
    const unsigned long long bal = __ballot(pr);
    const unsigned msk = half ? (unsigned)(bal >> 32) : (unsigned)bal;
    if (n > 0) {
      if (msk) {
        const int f = __builtin_ctz(msk);
        hi = lo + (int)(((long long)n * (f + 1)) / 33);
        if (f > 0) lo = lo + (int)(((long long)n * f) / 33) + 1;
      } else {
        lo = lo + (int)(((long long)n * 32) / 33) + 1;
      }
    }
  }
  s0 = __shfl(lo, 0, 64);
  s1 = __shfl(lo, 32, 64);
}
__global__ __launch_bounds__(256) void k_db_gather(lorb_ba_window_dev w, BaDev d, int K, const int* __restrict__ key,
                                                   const int* __restrict__ val, DbFused f, DbCams cams) {
  const int gt = blockIdx.x * 256 + threadIdx.x, gs = gridDim.x * 256;
  // the upload, from the mapped staging (PCIe reads, no copy launch before this kernel)
  for (int i = gt; i < f.up_words; i += gs) f.up_dst[i] = f.up_src[i];
  const int* __restrict__ perm = cams.perm;
  const int* __restrict__ gcam = cams.gcam;
  {  // initial values and camera activity
    const int m = max(max(6 * f.C, 6 * f.F), 3 * f.P);
    for (int i = gt; i < m; i += gs) {
      if (i < 6 * f.C) {
        const int c = i / 6, q = i - 6 * c;
        d.x_init_pose[6 * perm[c] + q] = (double)w.d_pose_init[i];
        if (q == 0) const_cast<int*>(d.cam_active)[perm[c]] = gcam[c] > 0;
      }
      if (i < 6 * f.F) const_cast<double*>(d.fixed_pose)[i] = (double)w.d_fixed_pose[i];
      if (i < 3 * f.P) d.x_init_pt[i] = (double)w.d_point_init[i];
    }
  }
  for (int g = gt >> 6; g < f.G; g += gs >> 6) {  // point groups, one wavefront each
    int s0, s1;
    group_bounds(d.pt_obs_off, f.P, (long long)g * f.S, (long long)(g + 1) * f.S, threadIdx.x & 63, s0, s1);
    if ((threadIdx.x & 63) == 0) {
      PBlk b;
      b.win = 0; b.p0 = s0; b.cnt = s1 - s0; b.o0 = d.pt_obs_off[s0]; b.no = d.pt_obs_off[s1] - d.pt_obs_off[s0];
      const_cast<PBlk*>(d.pblk)[g] = b;
    }
  }
  for (int i = gt; i < f.nsg; i += gs) f.sgrp[i] = make_int4(0, i * f.sgf, min(f.sgf, f.G - i * f.sgf), 0);
  for (int i = gt; i < f.env_n; i += gs) d.env_part[i] = 0.0;
  for (int i = gt; i < f.bits_n; i += gs) f.bits[i] = 0ull;
  for (int i = gt; i < f.cov_n; i += gs) f.cov[i] = 0;
  if (gt == 0) { f.hdr[1] = 0; f.hdr[2] = 0; }
  // the point-sorted observation records
  for (int e = gt; e < K; e += gs) {
    const int k = f.sorted ? e : val[e];
    const int fr = w.d_obs_frame[k];
    const_cast<int*>(d.obs_pt)[e] = f.sorted ? w.d_obs_point[e] : key[e];
    const_cast<int*>(d.obs_cam)[e] = fr >= 0 ? perm[fr] : -1;
    const_cast<int*>(d.obs_fix)[e] = fr >= 0 ? -1 : -1 - fr;
    const_cast<double2*>(d.obs_uv)[e] = make_double2(w.d_obs_uv[2 * k], w.d_obs_uv[2 * k + 1]);
  }
}

// plan camera order -> caller order, as float (Frame::SetPose / MapPoint::SetWorldPos write-back).
// ring (the LocalMapping map's keyframe ring of R slots): caller pose c goes to slot (t0 + c) mod R.
__global__ __launch_bounds__(256) void k_db_result(BaDev d, int C, int P, const int* __restrict__ perm,
                                                   float* __restrict__ pose_out, float* __restrict__ pt_out,
                                                   float* __restrict__ ring, int R, int t0) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  const int cur = d.st[0].cur;
  if ((pose_out || ring) && i < 6 * C) {
    const int c = i / 6, q = i - 6 * c;
    const float v = (float)d.x_pose[cur][6 * perm[c] + q];
    if (pose_out) pose_out[i] = v;
    if (ring) {
      const int r = (t0 + c) % R;
      ring[6 * (r < 0 ? r + R : r) + q] = v;
    }
  }
  if (pt_out)
    for (int k = i; k < 3 * P; k += gridDim.x * 256) pt_out[k] = (float)d.x_pt[cur][k];
}

// the same in double (the Ceres parameter blocks after Solve) plus the summary, into one buffer for
// one D2H copy: [poses 6C (caller order) | points 3P | iterations, successful steps, termination,
// initial cost, final cost]
__global__ __launch_bounds__(256) void k_db_result64(BaDev d, int C, int P, const int* __restrict__ perm,
                                                     double* __restrict__ out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  const WinState& st = d.st[0];
  const int cur = st.cur;
  if (i < 6 * C) {
    const int c = i / 6, q = i - 6 * c;
    out[i] = d.x_pose[cur][6 * perm[c] + q];
  }
  for (int k = i; k < 3 * P; k += gridDim.x * 256) out[6 * C + k] = d.x_pt[cur][k];
  if (i == 0) {
    double* s = out + 6 * C + 3 * P;
    s[0] = st.iter; s[1] = st.n_success; s[2] = st.term; s[3] = st.initial_cost; s[4] = st.cost;
  }
}

int dev_build_issue(lorb_ctx* ctx, const lorb_ba_window_dev* w, lorb_ba_plan* P, int* lerr_out);
int dev_build_finish(lorb_ctx* ctx, const lorb_ba_window_dev* w, lorb_ba_plan* P, int lerr);

}  // namespace

namespace lorb {
int ba_plan_update_dev_issue(lorb_ba_plan* P, const lorb_ba_window_dev* w) {
  if (!P || !w || !P->devb || P->comm) return LORB_E_INVALID;
  int lerr = 0;
  return dev_build_issue(P->ctx, w, P, &lerr);
}
int ba_plan_update_dev_finish(lorb_ba_plan* P, const lorb_ba_window_dev* w) {
  if (!P || !w || !P->devb || P->comm) return LORB_E_INVALID;
  return dev_build_finish(P->ctx, w, P, 0);
}

void ba_plan_sorted_hint(lorb_ba_plan* P, bool sorted) {
  if (P && P->devb) P->devb->sorted_hint = sorted;
}

const int* ba_plan_point_offsets(const lorb_ba_plan* P) { return P && P->devb ? P->dev.pt_obs_off : nullptr; }

void ba_plan_window_counts(const lorb_ba_plan* P, int* n_points, int* n_obs) {
  *n_points = P->Ptot;  // the live counts the last device build read back (its header)
  *n_obs = P->K;
}

int ba_plan_result_ring_dev(lorb_ba_plan* P, float* ring, int R, int t0, float* d_point_out) {
  if (!P || !P->devb || !ring || R < 1) return LORB_E_INVALID;
  const int C = P->Ctot, Pn = P->Ptot;
  const int m = std::max(std::max(6 * C, 1), std::min(3 * Pn, 256 * 1024));
  hipLaunchKernelGGL(k_db_result, dim3(lorb::ceil_div(m, 256)), dim3(256), 0, P->ctx->stream, P->dev, C, Pn,
                     P->devb->perm, (float*)nullptr, d_point_out, ring, R, t0);
  LORB_CHECK_LAUNCH(P->ctx);
  return LORB_OK;
}

int ba_plan_result64_dev(lorb_ba_plan* P, double* d_out) {
  if (!P || !P->devb || !d_out) return LORB_E_INVALID;
  const int C = P->Ctot, Pn = P->Ptot;
  const int m = std::max(std::max(6 * C, 1), std::min(3 * Pn, 256 * 1024));
  hipLaunchKernelGGL(k_db_result64, dim3(lorb::ceil_div(m, 256)), dim3(256), 0, P->ctx->stream, P->dev, C, Pn,
                     P->devb->perm, d_out);
  LORB_CHECK_LAUNCH(P->ctx);
  return LORB_OK;
}
}  // namespace lorb

namespace {

template <typename T, typename Cap>
int grow(lorb_ba_plan* P, T** ptr, Cap* cap, size_t need) {
  if (*ptr && (size_t)*cap >= need) return LORB_OK;
  if (*ptr) {
    LORB_HIP(P->ctx, hipStreamSynchronize(P->ctx->stream));
    LORB_HIP(P->ctx, hipFree(*ptr));
    auto it = std::find(P->allocs.begin(), P->allocs.end(), (void*)*ptr);
    if (it != P->allocs.end()) P->allocs.erase(it);
  }
  const size_t n = std::max<size_t>(need + need / 4, 16);
  LORB_TRY(dalloc(P, n, ptr));
  *cap = (Cap)n;
  P->has_graph = false;  // kernel arguments changed
  P->gen++;
  return LORB_OK;
}

// capacity allocations (once per plan)
int dev_alloc(lorb_ctx* ctx, const lorb_ba_window_dev* w, lorb_ba_plan* P) {
  lorb_ba_devbuild& b = *P->devb;
  b.K_cap = w->max_obs; b.P_cap = w->max_points; b.C = w->n_poses; b.F = w->n_fixed;
  b.Wd = (std::max(b.P_cap, 1) + 63) / 64;
  const size_t K = (size_t)std::max(b.K_cap, 1), Pn = (size_t)std::max(b.P_cap, 1), C = (size_t)std::max(b.C, 1);
  BaDev& d = P->dev;
  if (b.C > kPmSpan)
    return lorb::set_error(ctx, LORB_E_UNSUPPORTED, "device-built plans hold windows of <= %d cameras (%d)", kPmSpan, b.C);
  LORB_TRY(dalloc(P, K, &b.key_out)); LORB_TRY(dalloc(P, K, &b.val_out));
  {
    const size_t ints = ((Pn + 1 + 8 + C * C + C) + 1) & ~(size_t)1;  // the u64 bitsets 8-byte aligned
    b.scr_bytes = sizeof(int) * ints + sizeof(unsigned long long) * C * (size_t)b.Wd;
    unsigned char* m;
    LORB_TRY(dalloc(P, b.scr_bytes, &m));
    b.scr = reinterpret_cast<int*>(m);
    b.pt_cnt = b.scr; b.hdr = b.pt_cnt + Pn + 1; b.cov = b.hdr + 8; b.cam_cnt = b.cov + C * C;
    b.bits = reinterpret_cast<unsigned long long*>(b.scr + ints);
  }
  int *a_pt, *a_cam, *a_fix, *a_act, *a_ptoff;
  double2* a_uv;
  double* a_fixp;
  LORB_TRY(dalloc(P, K, &a_pt)); LORB_TRY(dalloc(P, K, &a_cam)); LORB_TRY(dalloc(P, K, &a_fix));
  LORB_TRY(dalloc(P, K, &a_uv)); LORB_TRY(dalloc(P, C, &a_act));
  LORB_TRY(dalloc(P, Pn + 1, &a_ptoff)); LORB_TRY(dalloc(P, (size_t)std::max(b.F, 1) * 6, &a_fixp));
  d.obs_pt = a_pt; d.obs_cam = a_cam; d.obs_fix = a_fix; d.obs_uv = a_uv;
  d.cam_active = a_act; d.pt_obs_off = a_ptoff; d.fixed_pose = a_fixp;
  LORB_TRY(dalloc(P, C * 6, &d.x_init_pose)); LORB_TRY(dalloc(P, Pn * 3, &d.x_init_pt));
  LORB_TRY(dalloc(P, C * 6, &d.x_pose[0])); LORB_TRY(dalloc(P, C * 6, &d.x_pose[1]));
  LORB_TRY(dalloc(P, Pn * 3, &d.x_pt[0])); LORB_TRY(dalloc(P, Pn * 3, &d.x_pt[1]));
  LORB_TRY(dalloc(P, C * 6, &d.scale_pose)); LORB_TRY(dalloc(P, Pn * 3, &d.scale_pt));
  LORB_TRY(dalloc(P, Pn * 3, &d.etb)); LORB_TRY(dalloc(P, Pn * 6, &d.pinv));
  // the solve block is rhs (n) | wfail (1) | pad | env (up to the dense n x n): rhs and wfail at fixed
  // places, so the captured solve survives a rebuild that changes the band, and a sharded plan's
  // exchange 2 is one contiguous all-reduce of x2_off + env_total doubles
  const size_t n = 6 * C, lin_n = C * 27 + 2, x2_off = (n + 1 + 31) & ~(size_t)31, solve_n = x2_off + n * n;
  lorb_comm* comm = P->comm;
  double *lin, *mx, *sol, *stp;
  // [lin | pad | solve] in one block, as in build_plan
  const size_t lin_pad = (lin_n + 31) & ~(size_t)31;
  LORB_TRY(dalloc(P, lin_pad + solve_n, &lin)); LORB_TRY(dalloc(P, (size_t)1, &mx));
  sol = lin + lin_pad;
  LORB_TRY(dalloc(P, (size_t)3, &stp));
  P->fx_n = lin_pad + solve_n;
  d.U = lin; d.V = lin + C * 21; d.wlin = lin + C * 27; d.wmax = mx;
  d.rhs = sol; d.wfail = sol + n; d.env = sol + x2_off;
  d.wstep = stp;
  P->x2_off = x2_off;
  b.sol_n = solve_n;
  // over one rank the exchanges are the identity: the partial buffers are the global ones (the
  // collectives then run in place, no copy)
  if (comm && comm->nranks > 1) {  // this rank's partial sums (see BaDev), all-reduced into the global buffers
    double *linp, *mxp, *solp, *stpp;
    LORB_TRY(dalloc(P, lin_pad + solve_n, &linp)); LORB_TRY(dalloc(P, (size_t)1, &mxp));
    solp = linp + lin_pad;
    LORB_TRY(dalloc(P, (size_t)3, &stpp));
    LORB_HIP(ctx, hipMemsetAsync(linp, 0, sizeof(double) * (lin_pad + solve_n), ctx->stream));
    d.U_part = linp; d.V_part = linp + C * 21; d.wlin_part = linp + C * 27; d.wmax_part = mxp;
    d.rhs_part = solp; d.wfail_part = solp + n; d.env_part = solp + x2_off;
    d.wstep_part = stpp;
    b.sol_part = solp;
  } else {
    d.U_part = d.U; d.V_part = d.V; d.wlin_part = d.wlin; d.wmax_part = d.wmax;
    d.rhs_part = d.rhs; d.wfail_part = d.wfail; d.env_part = d.env;
    d.wstep_part = d.wstep;
    b.sol_part = sol;
  }
  P->x2_send = b.sol_part; P->x2_recv = sol;
  d.sharded = comm ? 1 : 0;
  d.rank0 = comm ? (comm->rank == 0) : 1;
  LORB_TRY(dalloc(P, C, &d.rot_lin)); LORB_TRY(dalloc(P, C, &d.rot_cand));
  LORB_TRY(dalloc(P, (size_t)std::max(b.F, 1), &d.rot_fix)); LORB_TRY(dalloc(P, (size_t)std::max(b.F, 1), &d.rotv_fix));
  LORB_TRY(dalloc(P, n, &d.ycam));
#ifdef LORB_CHOL_TRACE
  LORB_TRY(dalloc(P, (size_t)512, &d.dbg));
#elif defined(LORB_LS_STAMPS)
  LORB_TRY(dalloc(P, (K + Pn + 1) * 8, &d.dbg));  // >= 8 per point group at any build
#else
  LORB_TRY(dalloc(P, (size_t)8, &d.dbg));
#endif
  LORB_TRY(dalloc(P, ((size_t)n / 16 + 2) * 1024, &d.kco));
  LORB_TRY(dalloc(P, (size_t)1, &P->d_state)); d.st = P->d_state;
  LORB_TRY(dalloc(P, (size_t)LORB_LM_TRACE_CAP, &d.trace));
  P->W = 1;
  P->hwin.assign(1, BaWin{});
  P->pt_launch = b.P_cap;
  return LORB_OK;
}

// (re)allocate the upload block for bp_need block pairs; repoints BaDev at it
int up_alloc(lorb_ba_plan* P, int bp_need) {
  lorb_ba_devbuild& b = *P->devb;
  if (b.up_dev && b.up_bp_cap >= bp_need) return LORB_OK;
  lorb_ctx* ctx = P->ctx;
  const int cap = std::max(bp_need + bp_need / 4, 16);
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  const size_t C = (size_t)std::max(b.C, 1);
  b.off_live = al(sizeof(BaWin));
  b.off_perm = b.off_live + 256;
  b.off_gcam = b.off_perm + al(4 * C);
  b.off_bp = b.off_gcam + al(4 * C);
  b.up_bytes = b.off_bp + sizeof(BlockPair) * (size_t)cap;
  if (b.up_dev) {
    LORB_HIP(ctx, hipStreamSynchronize(ctx->stream));
    LORB_HIP(ctx, hipFree(b.up_dev));
    auto it = std::find(P->allocs.begin(), P->allocs.end(), (void*)b.up_dev);
    if (it != P->allocs.end()) P->allocs.erase(it);
    (void)hipHostFree(b.up_host);
    b.up_host = nullptr;
  }
  LORB_TRY(dalloc(P, b.up_bytes, &b.up_dev));
  LORB_HIP(ctx, hipHostMalloc(reinterpret_cast<void**>(&b.up_host), b.up_bytes));
  {
    void* hd = nullptr;
    LORB_HIP(ctx, hipHostGetDevicePointer(&hd, b.up_host, 0));
    b.up_host_dev = static_cast<const unsigned char*>(hd);
  }
  b.up_bp_cap = cap;
  BaDev& d = P->dev;
  d.win = reinterpret_cast<const BaWin*>(b.up_dev);
  d.live = reinterpret_cast<const int*>(b.up_dev + b.off_live);
  b.perm = reinterpret_cast<int*>(b.up_dev + b.off_perm);
  b.gcam = reinterpret_cast<int*>(b.up_dev + b.off_gcam);
  d.bp = reinterpret_cast<const BlockPair*>(b.up_dev + b.off_bp);
  P->grid_bp = cap;
  P->has_graph = false;
  P->gen++;
  return LORB_OK;
}

// phase 1 of a build on the ctx stream: per-point counts, camera x point bitsets, point offsets,
// the counting sort by point when the slots are not sorted, covisibility counts; then the one
// readback (hdr | cov | cam_cnt are contiguous in the scratch: one copy) and an event behind it.
// The scratch is left clear by the previous build's k_db_gather; only a build that stopped before it
// (an error) leaves it dirty.
int db_phase1_issue(lorb_ctx* ctx, const lorb_ba_window_dev* w, lorb_ba_plan* P, bool sorted) {
  lorb_ba_devbuild& b = *P->devb;
  hipStream_t s = ctx->stream;
  BaDev& d = P->dev;
  const int C = b.C, F = b.F, Kc = w->max_obs;
  const size_t nrb = 8 + (size_t)C + (size_t)C * C;
  const int nb_obs = lorb::ceil_div(std::max(Kc, 1), 256), nb_pt = lorb::ceil_div(std::max(b.P_cap, 1), 256);
  if (b.pinned_n < nrb) {
    if (b.pinned) (void)hipHostFree(b.pinned);
    b.pinned = nullptr; b.pinned_n = 0;
    LORB_HIP(ctx, hipHostMalloc(reinterpret_cast<void**>(&b.pinned), sizeof(int) * nrb));
    b.pinned_n = nrb;
  }
  if (!b.rb_ev) LORB_HIP(ctx, hipEventCreateWithFlags(&b.rb_ev, hipEventDisableTiming));
  if (b.dirty) LORB_HIP(ctx, hipMemsetAsync(b.scr, 0, b.scr_bytes, s));
  b.dirty = true;
  const bool fuse = sorted && C > 0 && sizeof(int) * ((size_t)C * C + C) <= (size_t)kDbFuseLds;
  if (sorted) {
    const size_t lds = sizeof(unsigned long long) * kDbWords * std::max(C, 1) +
                       (fuse ? sizeof(int) * ((size_t)C * C + C) : 0);
    if (fuse)
      hipLaunchKernelGGL(k_db_sorted<true>, dim3(lorb::ceil_div(Kc + 1, 256)), dim3(256), lds, s, *w, C, F, b.Wd,
                         const_cast<int*>(d.pt_obs_off), b.hdr, b.bits, b.cov, b.cam_cnt);
    else
      hipLaunchKernelGGL(k_db_sorted<false>, dim3(lorb::ceil_div(Kc + 1, 256)), dim3(256), lds, s, *w, C, F, b.Wd,
                         const_cast<int*>(d.pt_obs_off), b.hdr, b.bits, b.cov, b.cam_cnt);
  } else {
    hipLaunchKernelGGL(k_db_keys, dim3(nb_obs), dim3(256), 0, s, *w, C, F, b.Wd, b.pt_cnt, b.hdr, b.bits);
    hipLaunchKernelGGL(k_db_scan1, dim3(1), dim3(1024), 0, s, b.pt_cnt, const_cast<int*>(d.pt_obs_off), b.P_cap + 1,
                       w->d_n_points, b.hdr);
    if (Kc > 0) {
      hipLaunchKernelGGL(k_db_scatter, dim3(nb_obs), dim3(256), 0, s, *w, C, F, d.pt_obs_off, b.pt_cnt, b.val_out);
      hipLaunchKernelGGL(k_db_segsort, dim3(nb_pt), dim3(256), 0, s, *w, d.pt_obs_off, b.val_out, b.key_out);
    }
  }
  if (C > 0 && !fuse)
    hipLaunchKernelGGL(k_db_cov, dim3(lorb::ceil_div(C * (C + 1) / 2, 4)), dim3(256), 0, s, C, b.Wd, b.bits, b.cov,
                       b.cam_cnt);
  LORB_CHECK_LAUNCH(ctx);
  LORB_HIP(ctx, hipMemcpyAsync(b.pinned, b.hdr, sizeof(int) * nrb, hipMemcpyDeviceToHost, s));
  LORB_HIP(ctx, hipEventRecord(b.rb_ev, s));
  b.rb_sorted = sorted;
  b.rb_fuse = fuse;
  b.rb_pending = true;
  return LORB_OK;
}

// the readback of an issued phase 1 landed (polled); slots found out of order on the sorted path
// (or unused) rerun the general phase from a cleared scratch
int db_phase1_wait(lorb_ctx* ctx, const lorb_ba_window_dev* w, lorb_ba_plan* P) {
  lorb_ba_devbuild& b = *P->devb;
  for (;;) {
    b.rb_pending = false;
    LORB_HIP(ctx, lorb::spin_wait(b.rb_ev));
    if (!(b.rb_sorted && (b.pinned[2] & 16))) return LORB_OK;
    b.sorted_hint = false;
    LORB_TRY(db_phase1_issue(ctx, w, P, false));
  }
}

// the first half of a build: the shape check and phase 1 with its readback queued (no wait).  A
// rank-local failure of a sharded plan is kept for dev_build_finish (see there).
int dev_build_issue(lorb_ctx* ctx, const lorb_ba_window_dev* w, lorb_ba_plan* P, int* lerr_out) {
  lorb_ba_devbuild& b = *P->devb;
  const bool shape_ok = w->n_poses == b.C && w->n_fixed == b.F && w->max_obs <= b.K_cap && w->max_points <= b.P_cap;
  *lerr_out = shape_ok ? 0 : 32;
  if (!shape_ok && !P->comm)
    return lorb::set_error(ctx, LORB_E_INVALID, "window shape differs from the plan's (cameras %d/%d, fixed %d/%d)",
                           w->n_poses, b.C, w->n_fixed, b.F);
  if (!shape_ok) return LORB_OK;
  const int rc = db_phase1_issue(ctx, w, P, b.sorted_hint);
  if (rc != LORB_OK && P->comm) { *lerr_out |= 64; return LORB_OK; }
  return rc;
}

int dev_build_finish(lorb_ctx* ctx, const lorb_ba_window_dev* w, lorb_ba_plan* P, int lerr);

// a whole build: dev_build_issue + dev_build_finish
int dev_build(lorb_ctx* ctx, const lorb_ba_window_dev* w, lorb_ba_plan* P) {
  int lerr = 0;
  LORB_TRY(dev_build_issue(ctx, w, P, &lerr));
  return dev_build_finish(ctx, w, P, lerr);
}

// the second half: wait for the readback, then the host phase and the structure kernel.
// Sharded plans are collective: a rank-local failure before the exchange below (a shape that
// differs from the plan's, a failed allocation or copy) is not returned here -- it becomes an
// error bit of the all-reduce, so every rank reaches the exchange and every rank returns the error.
int dev_build_finish(lorb_ctx* ctx, const lorb_ba_window_dev* w, lorb_ba_plan* P, int lerr) {
  lorb_ba_devbuild& b = *P->devb;
  const bool shape_ok = !(lerr & 32);
  hipStream_t s = ctx->stream;
  BaDev& d = P->dev;
  const int C = b.C, F = b.F;
  const size_t nrb = 8 + (size_t)C + (size_t)C * C;
  const int phase_rc = (lerr || !b.rb_pending) ? LORB_OK : db_phase1_wait(ctx, w, P);
  const bool sorted = b.rb_sorted, fuse = b.rb_fuse;
  static const bool hp_log = [] { const char* e = getenv("LORB_HOST_PHASE"); return e && e[0] == '1'; }();
  const auto hp_t0 = std::chrono::steady_clock::now();
  auto hp_last = hp_t0;
  auto hp_mark = [&](int k) {
    if (!hp_log) return;
    const auto now = std::chrono::steady_clock::now();
    P->hp_sec[k] += std::chrono::duration<double, std::micro>(now - hp_last).count();
    hp_last = now;
  };
  if (phase_rc != LORB_OK) {
    if (!P->comm) return phase_rc;
    lerr |= 64;
  }
  // the readback landed by DMA: none of its lines are in the CPU's caches.  One sequential copy
  // (prefetched) into a reused host buffer, then the column-wise triangle fill and the scans below
  // run on cached data instead of one DRAM round trip per line touched out of order.
  b.h_copy.resize(nrb);
  if (lerr) std::fill(b.h_copy.begin(), b.h_copy.end(), 0);  // a failed rank contributes an empty structure
  else std::memcpy(b.h_copy.data(), b.pinned, sizeof(int) * nrb);
  int* H = b.h_copy.data();
  if (fuse)  // k_db_sorted<true> filled the lower triangle
    for (int i = 0; i < C; ++i)
      for (int j = i + 1; j < C; ++j) H[8 + (size_t)i * C + j] = H[8 + (size_t)j * C + i];
  const int K = H[0], maxk = H[1], err = H[2], Pn = H[3];
  const int* cov = H + 8;
  const int* cam_cnt = H + 8 + (size_t)C * C;
  // sharded: the camera-level structure is global -- sum the ranks' covisibility and camera counts
  // (camera order, band and camera activity must agree on every rank) and their error flags (every
  // rank returns the same error, so none is left waiting in a later collective)
  const int* gcov = cov;
  const int* gcam = cam_cnt;
  int K_all = K, gerr = err, gmaxk = maxk;
  std::vector<int> g_int;
  if (P->comm) {
    // [cov | cam_cnt (contiguous, m) | K | n_points out of range | error bits 0..6] summed; the largest
    // per-point count (the group size check) by a max
    const size_t m = (size_t)C * C + C;
    b.h_red.assign(m + 9, 0.0);
    for (size_t i = 0; i < m; ++i) b.h_red[i] = (double)cov[i];
    b.h_red[m] = K;
    b.h_red[m + 1] = (Pn < 0 || Pn > b.P_cap) ? 1.0 : 0.0;
    for (int q = 0; q < 7; ++q) b.h_red[m + 2 + q] = ((err | lerr) >> q) & 1;
    LORB_TRY(lorb::comm_allreduce_host(P->comm, b.h_red.data(), b.h_red.size(), LORB_OP_SUM));
    double mk = maxk;
    LORB_TRY(lorb::comm_allreduce_host(P->comm, &mk, 1, LORB_OP_MAX));
    g_int.resize(m);
    for (size_t i = 0; i < m; ++i) g_int[i] = (int)b.h_red[i];
    gcov = g_int.data();
    gcam = g_int.data() + (size_t)C * C;
    K_all = (int)b.h_red[m];
    gerr = b.h_red[m + 1] > 0.0 ? 16 : 0;
    for (int q = 0; q < 7; ++q) gerr |= b.h_red[m + 2 + q] > 0.0 ? 1 << q : 0;
    gmaxk = (int)mk;
  }
  if (gerr & 32)
    return lorb::set_error(ctx, LORB_E_INVALID, "window shape differs from the plan's on %s (cameras %d/%d, fixed %d/%d)",
                           shape_ok ? "another rank" : "this rank", w->n_poses, b.C, w->n_fixed, b.F);
  if (gerr & 64)
    return phase_rc != LORB_OK ? phase_rc
                               : lorb::set_error(ctx, LORB_E_DEVICE, "device plan build failed on another rank");
  // a count beyond capacity first: the slots read up to the capacity then hold no real observations
  if (gerr & 8) return lorb::set_error(ctx, LORB_E_INVALID, "live point / observation count outside [0, capacity] (%d / %d)",
                                       b.P_cap, b.K_cap);
  if (gerr & 1) return lorb::set_error(ctx, LORB_E_INVALID, "observation with a point index outside [0, n_points)");
  if (gerr & 2) return lorb::set_error(ctx, LORB_E_INVALID, "observation with a frame index >= n_poses");
  if (gerr & 4) return lorb::set_error(ctx, LORB_E_INVALID, "a point observed twice by one camera");
  if ((gerr & 16) || Pn < 0 || Pn > b.P_cap) return lorb::set_error(ctx, LORB_E_INVALID, "n_points %d outside [0, %d]", Pn, b.P_cap);
  if (kGB - gmaxk < 1)
    return lorb::set_error(ctx, LORB_E_UNSUPPORTED, "a point with %d observations (device plans hold <= %d)", gmaxk, kGB - 1);
  hp_mark(0);
  // 3. host: camera order, blocks, band, groups (order, band, activity from the global structure;
  //    the block pair lists from this rank's observations)
  // the camera order depends only on the adjacency pattern: compared in place against the last
  // build's (no allocation on the step's host phase), recomputed when it changed
  bool same_adj = b.last_adj.size() == (size_t)C * C;
  for (int i = 0; i < C && same_adj; ++i) {
    const int* row = gcov + (size_t)i * C;
    const char* last = b.last_adj.data() + (size_t)i * C;
    for (int j = 0; j < C; ++j)
      if (last[j] != (char)((i == j && gcam[i] > 0) || row[j] > 0)) { same_adj = false; break; }
  }
  if (!same_adj) {
    std::vector<char> adj((size_t)C * C, 0);
    for (int i = 0; i < C; ++i)
      for (int j = 0; j < C; ++j) adj[(size_t)i * C + j] = (i == j && gcam[i] > 0) || gcov[(size_t)i * C + j] > 0;
    b.last_map = camera_order(C, adj);
    b.last_adj.swap(adj);
  }
  const std::vector<int>& map = b.last_map;
  hp_mark(1);
  std::vector<int> inv(C);
  for (int c = 0; c < C; ++c) inv[map[c]] = c;
  P->cam_map.assign(1, map);
  std::vector<BlockPair> bps;
  std::vector<int> fc(C);
  int n_pairs = 0;
  for (int ch = 0; ch < C; ++ch) {  // std::map order of the host builder: (ch, cl) ascending
    fc[ch] = ch;
    for (int cl = 0; cl <= ch; ++cl) {
      const int cnt = ch == cl ? cam_cnt[inv[ch]] : cov[(size_t)inv[ch] * C + inv[cl]];
      if (ch != cl && gcov[(size_t)inv[ch] * C + inv[cl]] > 0) fc[ch] = std::min(fc[ch], cl);
      if (ch != cl && cnt == 0) continue;
      bps.push_back(BlockPair{0, ch, cl, n_pairs, cnt});
      n_pairs += cnt;
    }
  }
  const int n = 6 * C;
  int bwid = 0;
  for (int c = 0; c < C; ++c) bwid = std::max(bwid, 6 * c + 5 - 6 * fc[c]);
  if (n == 0) bwid = 0;
  const int S = kGB - (maxk + 1) + 1;  // >= 1 (checked above)
  const int G = Pn > 0 ? (K + Pn - 1) / S + 1 : 0;
  BaWin bw{};
  bw.pose_base = 0; bw.n_poses = C; bw.point_base = 0; bw.n_points = Pn; bw.pblk_base = 0; bw.n_pblk = G;
  bw.env_base = 0; bw.env_size = n * (bwid + 1); bw.n = n; bw.row_base = 0; bw.bw = bwid;
  bw.obs_base = 0; bw.n_obs = K; bw.n_obs_all = K_all;
  bw.fx = w->fx; bw.fy = w->fy; bw.cx = w->cx; bw.cy = w->cy;
  const int SF = sg_factor(G), NSG = G > 0 ? (G + SF - 1) / SF : 0;  // partial runs (k_db_gather fills them)
  bw.sg_base = 0; bw.n_sg = NSG;
  long long part_total = 0;
  pm_layout(bw, C, part_total);  // a group (or run) spans at most the window's C <= kPmSpan cameras
  LORB_TRY(part_budget_check(ctx, part_total));
  P->hwin[0] = bw;
  P->Ctot = C; P->Ptot = Pn; P->K = K; P->NF = F; P->n_pblk = G; P->n_bp = (int)bps.size(); P->n_pairs = n_pairs;
  P->env_total = bw.env_size; P->n_total = n;
  P->max_env = bw.env_size + 2 * n; P->max_bw = bwid;
  P->min_bw = n > 0 ? bwid : (1 << 30);
  {
    // the Cholesky's LDS is sized for a band of 48 (the widest k_ba_chol_w / _2s take) when that
    // fits, so that a narrower band after a rebuild keeps the captured solve
    const int n16 = (n + 15) & ~15;
    auto env_w = [&](int bwv) {
      return std::max(std::max(n16 * (bwv + 1) + 2 * n16 + 64 * 18, (n16 + 48) * (bwv + 2) + 2 * 64 * 18 + 48),
                      chol2s_words(n16, bwv));
    };
    P->max_env_w = env_w(bwid);
    if (bwid <= 48 && sizeof(double) * (size_t)env_w(48) <= (size_t)kLdsBudget) P->max_env_w = env_w(48);
    P->min_n16 = n16 > 0 ? n16 : (1 << 30);
  }
  hp_mark(2);
  // grow-only structure buffers; the point-group kernels launch at capacity
  PBlk* pb = const_cast<PBlk*>(d.pblk);
  LORB_TRY(grow(P, &pb, &b.pblk_cap, (size_t)std::max(G, 1)));
  d.pblk = pb;
  {
    double* pt = d.part;
    LORB_TRY(grow(P, &pt, &b.part_cap, (size_t)b.pblk_cap * 8));
    d.part = pt;
  }
  P->grid_pblk = b.pblk_cap;
  {  // group partials (grow-only; a reallocation re-captures the LM graph)
    LORB_TRY(grow(P, &d.gpart, &b.gpart_cap, (size_t)std::max(part_total, 1ll)));
    int2* gsp = d.gspan;
    LORB_TRY(grow(P, &gsp, &b.gspan_cap, (size_t)b.pblk_cap));
    d.gspan = gsp;
    int4* sgp = const_cast<int4*>(d.sgrp);
    LORB_TRY(grow(P, &sgp, &b.sgrp_cap, (size_t)b.pblk_cap));
    d.sgrp = sgp;
  }
  P->has_super = SF > 1;
  P->grid_sg = b.pblk_cap;  // runs <= groups: launched at the groups' capacity, live[2] in use
  LORB_TRY(up_alloc(P, (int)bps.size()));
  hp_mark(3);
  // one upload (pinned staging, stream-ordered; the next build writes the staging only after its
  // own readback synchronised the stream).  No copy launch: k_db_gather copies the staging over the
  // bus and takes the camera tables as kernel arguments (the step's host phase ends with the
  // gather's launch)
  int up_words = 0;
  {
    unsigned char* h = b.up_host;
    memcpy(h, &P->hwin[0], sizeof(BaWin));
    const int live[3] = {G, (int)bps.size(), NSG};
    memcpy(h + b.off_live, live, sizeof(live));
    memcpy(h + b.off_perm, map.data(), sizeof(int) * C);
    memcpy(h + b.off_gcam, gcam, sizeof(int) * C);
    if (!bps.empty()) memcpy(h + b.off_bp, bps.data(), sizeof(BlockPair) * bps.size());
    const size_t bytes = b.off_bp + sizeof(BlockPair) * bps.size();
    up_words = (int)((bytes + 3) / 4);
  }
  hp_mark(4);
  // 4. structure kernel: gather (point-sorted observation records, initial values, point groups,
  //    the zeros the next build starts from)
  const int NB = lorb::ceil_div(K, 256);
  {
    // this rank's band starts from zeros (blocks it has no pairs of stay zero; sharded: the
    // all-reduce writes the global band every iteration)
    DbFused f{C, F, Pn, G, S, P->env_total, C * b.Wd, sorted ? 1 : 0, b.bits, b.hdr, b.cov, C * C + C,
              reinterpret_cast<const int*>(b.up_host_dev), reinterpret_cast<int*>(b.up_dev), up_words};
    f.sgf = SF; f.nsg = NSG; f.sgrp = const_cast<int4*>(d.sgrp);
    DbCams cams;
    for (int c = 0; c < C; ++c) { cams.perm[c] = map[c]; cams.gcam[c] = gcam[c]; }
    hipLaunchKernelGGL(k_db_gather, dim3(std::max(NB, 1)), dim3(256), 0, s, *w, d, K, b.key_out, b.val_out, f, cams);
    b.dirty = false;
    if (hp_log) {
      hp_mark(5);
      P->hp_us += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - hp_t0).count();
      P->hp_n++;
    }
  }
  LORB_CHECK_LAUNCH(ctx);
  return LORB_OK;
}

}  // namespace

extern "C" {

int lorb_ba_plan_create(lorb_ctx* ctx, int32_t n_windows, const lorb_ba_window* windows,
                        lorb_ba_plan** out) {
  if (!ctx || !out || n_windows < 0 || (n_windows > 0 && !windows)) return LORB_E_INVALID;
  *out = nullptr;
  lorb_ba_plan* P = new (std::nothrow) lorb_ba_plan();
  if (!P) return LORB_E_NOMEM;
  int rc = build_plan(ctx, n_windows, windows, P);
  if (rc != LORB_OK) { delete P; return rc; }
  *out = P;
  return LORB_OK;
}

int lorb_ba_plan_create_sharded(lorb_ctx* ctx, lorb_comm* comm, int32_t n_windows,
                                const lorb_ba_window* shards, lorb_ba_plan** out) {
  if (!ctx || !comm || !out || n_windows < 0 || (n_windows > 0 && !shards)) return LORB_E_INVALID;
  if (comm->ctx != ctx) return lorb::set_error(ctx, LORB_E_INVALID, "communicator belongs to another context");
  *out = nullptr;
  lorb_ba_plan* P = new (std::nothrow) lorb_ba_plan();
  if (!P) return LORB_E_NOMEM;
  P->comm = comm;
  int rc = build_plan(ctx, n_windows, shards, P);
  if (rc != LORB_OK) { delete P; return rc; }
  *out = P;
  return LORB_OK;
}

int lorb_ba_plan_create_dev(lorb_ctx* ctx, const lorb_ba_window_dev* win, lorb_ba_plan** out) {
  if (!ctx || !win || !out || win->n_poses < 0 || win->n_fixed < 0 || win->max_points < 0 || win->max_obs < 0 ||
      !win->d_n_points || !win->d_n_obs || (win->n_poses > 0 && !win->d_pose_init) ||
      (win->n_fixed > 0 && !win->d_fixed_pose) || (win->max_points > 0 && !win->d_point_init) ||
      (win->max_obs > 0 && (!win->d_obs_point || !win->d_obs_frame || !win->d_obs_uv)))
    return LORB_E_INVALID;
  *out = nullptr;
  lorb_ba_plan* P = new (std::nothrow) lorb_ba_plan();
  if (!P) return LORB_E_NOMEM;
  P->ctx = ctx;
  P->devb = new (std::nothrow) lorb_ba_devbuild();
  // slots sorted by point take k_db_sorted (no counting sort); unsorted ones fall back once and the
  // plan keeps the general path from then on
  if (P->devb) P->devb->sorted_hint = true;
  int rc = P->devb ? dev_alloc(ctx, win, P) : LORB_E_NOMEM;
  if (rc == LORB_OK) rc = dev_build(ctx, win, P);
  if (rc != LORB_OK) { delete P; return rc; }
  *out = P;
  return LORB_OK;
}

int lorb_ba_plan_create_sharded_dev(lorb_ctx* ctx, lorb_comm* comm, const lorb_ba_window_dev* shard,
                                    lorb_ba_plan** out) {
  if (!ctx || !comm || !shard || !out) return LORB_E_INVALID;
  if (comm->ctx != ctx) return lorb::set_error(ctx, LORB_E_INVALID, "communicator belongs to another context");
  if (shard->n_poses < 0 || shard->n_fixed < 0 || shard->max_points < 0 || shard->max_obs < 0 || !shard->d_n_points ||
      !shard->d_n_obs || (shard->n_poses > 0 && !shard->d_pose_init) || (shard->n_fixed > 0 && !shard->d_fixed_pose) ||
      (shard->max_points > 0 && !shard->d_point_init) ||
      (shard->max_obs > 0 && (!shard->d_obs_point || !shard->d_obs_frame || !shard->d_obs_uv)))
    return LORB_E_INVALID;
  *out = nullptr;
  lorb_ba_plan* P = new (std::nothrow) lorb_ba_plan();
  if (!P) return LORB_E_NOMEM;
  P->ctx = ctx;
  P->comm = comm;
  P->devb = new (std::nothrow) lorb_ba_devbuild();
  if (P->devb) P->devb->sorted_hint = true;  // as lorb_ba_plan_create_dev (shard.shard_window sorts by point)
  int rc = P->devb ? dev_alloc(ctx, shard, P) : LORB_E_NOMEM;
  if (rc == LORB_OK) rc = dev_build(ctx, shard, P);
  if (rc != LORB_OK) { delete P; return rc; }
  *out = P;
  return LORB_OK;
}

int lorb_ba_plan_update_dev(lorb_ba_plan* plan, const lorb_ba_window_dev* win) {
  if (!plan || !win) return LORB_E_INVALID;
  if (!plan->devb) return lorb::set_error(plan->ctx, LORB_E_INVALID, "not a device-built plan");
  return dev_build(plan->ctx, win, plan);
}

int lorb_ba_plan_result_dev(lorb_ba_plan* plan, float* d_pose_out, float* d_point_out) {
  if (!plan) return LORB_E_INVALID;
  if (!plan->devb) return lorb::set_error(plan->ctx, LORB_E_INVALID, "not a device-built plan");
  const int C = plan->Ctot, Pn = plan->Ptot;
  const int m = std::max(6 * C, std::min(3 * Pn, 256 * 1024));
  if (m > 0)
    hipLaunchKernelGGL(k_db_result, dim3(lorb::ceil_div(m, 256)), dim3(256), 0, plan->ctx->stream, plan->dev, C, Pn,
                       plan->devb->perm, d_pose_out, d_point_out, (float*)nullptr, 1, 0);
  LORB_CHECK_LAUNCH(plan->ctx);
  return LORB_OK;
}

int lorb_ba_plan_solve(lorb_ba_plan* plan, const lorb_lm_options* opt) {
  if (!plan || !opt) return LORB_E_INVALID;
  if (plan->W == 0) return LORB_OK;
  return plan_solve(plan, opt);
}

int lorb_ba_plan_read(lorb_ba_plan* plan, double* const* pose_out, double* const* point_out,
                      lorb_ba_summary* summaries) {
  if (!plan) return LORB_E_INVALID;
  if (plan->W == 0) return LORB_OK;
  return plan_read(plan, pose_out, point_out, summaries);
}

int lorb_ba_plan_trace(lorb_ba_plan* plan, int32_t window, lorb_lm_iteration* out, int32_t cap, int32_t* n_out) {
  if (!plan || !n_out || cap < 0 || (cap > 0 && !out)) return LORB_E_INVALID;
  *n_out = 0;
  if (window < 0 || window >= std::max(plan->W, 0)) return plan->W == 0 ? LORB_OK : LORB_E_INVALID;
  lorb_ctx* ctx = plan->ctx;
  WinState st;
  LORB_HIP(ctx, hipMemcpyAsync(&st, plan->d_state + window, sizeof(WinState), hipMemcpyDeviceToHost, ctx->stream));
  LORB_HIP(ctx, hipStreamSynchronize(ctx->stream));
  const int n = std::min(std::min(st.iter, (int)LORB_LM_TRACE_CAP), (int)cap);
  if (n > 0) {
    LORB_HIP(ctx, hipMemcpyAsync(out, plan->dev.trace + (size_t)window * LORB_LM_TRACE_CAP, sizeof(lorb_lm_iteration) * n,
                                 hipMemcpyDeviceToHost, ctx->stream));
    LORB_HIP(ctx, hipStreamSynchronize(ctx->stream));
  }
  *n_out = std::max(n, 0);
  return LORB_OK;
}

// diagnostic: copy the Cholesky phase stamps of window 0 (LORB_CHOL_STAMPS builds)
int lorb_ba_plan_debug_stamps(lorb_ba_plan* plan, unsigned long long* out8) {
  if (!plan || !out8) return LORB_E_INVALID;
#ifdef LORB_CHOL_TRACE
  const size_t nst = 512;  // trace builds: the caller passes 512 entries
#elif defined(LORB_LS_STAMPS)
  const size_t nst = (size_t)std::max(plan->n_pblk, plan->W) * 8;  // host-built plans: 8 per point group
#else
  const size_t nst = 8;
#endif
  LORB_HIP(plan->ctx, hipMemcpyAsync(out8, plan->dev.dbg, nst * sizeof(unsigned long long), hipMemcpyDeviceToHost, plan->ctx->stream));
  LORB_HIP(plan->ctx, hipStreamSynchronize(plan->ctx->stream));
  return LORB_OK;
}

int lorb_ba_plan_info(lorb_ba_plan* plan, int32_t* info, int32_t n) {
  if (!plan || !info || n < 0) return LORB_E_INVALID;
  int bw = 0;
  for (const BaWin& w : plan->hwin) bw = std::max(bw, w.bw);
  int reordered = 0;
  for (const auto& m : plan->cam_map)
    for (size_t c = 0; c < m.size(); ++c) reordered |= m[c] != (int)c;
  int runs = 0;
  for (const BaWin& w : plan->hwin) runs += w.n_sg;
  const int32_t v[11] = {bw, plan->chol_kind, plan->n_bp, plan->n_pblk, plan->K, plan->Ptot, plan->Ctot, reordered,
                         1, red_threads(plan), plan->has_super ? runs : 0};
  for (int i = 0; i < n && i < 11; ++i) info[i] = v[i];
  return LORB_OK;
}

int lorb_ba_plan_destroy(lorb_ba_plan* plan) {
  if (!plan) return LORB_OK;
  if (plan->ctx) (void)hipStreamSynchronize(plan->ctx->stream);
  delete plan;
  return LORB_OK;
}

int lorb_ba_group_create(lorb_ctx* ctx, int32_t n_plans, lorb_ba_plan* const* plans, lorb_ba_group** out) {
  if (!ctx || !out || n_plans < 1 || !plans) return LORB_E_INVALID;
  *out = nullptr;
  for (int k = 0; k < n_plans; ++k) {
    if (!plans[k]) return lorb::set_error(ctx, LORB_E_INVALID, "lorb_ba_group_create: plan %d is null", k);
    if (plans[k]->ctx != ctx)
      return lorb::set_error(ctx, LORB_E_INVALID, "lorb_ba_group_create: plan %d belongs to another context", k);
    for (int j = 0; j < k; ++j)
      if (plans[j] == plans[k]) return lorb::set_error(ctx, LORB_E_INVALID, "lorb_ba_group_create: plan %d appears twice", k);
  }
  lorb_ba_group* G = new (std::nothrow) lorb_ba_group();
  if (!G) return LORB_E_NOMEM;
  G->ctx = ctx;
  G->plans.assign(plans, plans + n_plans);
  *out = G;
  return LORB_OK;
}

int lorb_ba_group_solve(lorb_ba_group* group, const lorb_lm_options* opt) {
  if (!group || !opt) return LORB_E_INVALID;
  return group_solve(group, opt);
}

int lorb_ba_group_info(lorb_ba_group* group, int32_t* info, int32_t n) {
  if (!group || !info || n < 0) return LORB_E_INVALID;
  const int32_t v[3] = {(int32_t)group->plans.size(), group->n_fused, group->n_captures};
  for (int i = 0; i < n && i < 3; ++i) info[i] = v[i];
  return LORB_OK;
}

int lorb_ba_group_destroy(lorb_ba_group* group) {
  if (!group) return LORB_OK;
  (void)hipStreamSynchronize(group->ctx->stream);
  delete group;
  return LORB_OK;
}

int lorb_ba_local(lorb_ctx* ctx, int32_t n_windows, const lorb_ba_window* windows,
                  const lorb_lm_options* opt, double* const* pose_out, double* const* point_out,
                  lorb_ba_summary* summaries) {
  if (!ctx || !opt) return LORB_E_INVALID;
  lorb_ba_plan* P = nullptr;
  LORB_TRY(lorb_ba_plan_create(ctx, n_windows, windows, &P));
  int rc = lorb_ba_plan_solve(P, opt);
  if (rc == LORB_OK) rc = lorb_ba_plan_read(P, pose_out, point_out, summaries);
  lorb_ba_plan_destroy(P);
  return rc;
}

int lorb_ba_pose_only(lorb_ctx* ctx, const lorb_pose_problem_batch* prob,
                      const lorb_lm_options* opt, double* pose_out, float* Tcw_out,
                      lorb_ba_summary* summaries) {
  if (!ctx || !prob || !opt || !pose_out) return LORB_E_INVALID;
  const int nf = prob->n_frames;
  if (nf <= 0) return LORB_OK;
  const int nr = prob->res_off[nf];
  // every input in one pinned staging, poses and summaries stored straight into pinned memory.  A
  // batch whose frames all fit the kernel's register-resident residuals reads each input once: the
  // kernel then reads the mapped staging directly (no pull launch); larger frames re-read theirs
  // every pass, from HBM after a pull.
  int max_res = 0;
  for (int f = 0; f < nf; ++f) max_res = std::max(max_res, prob->res_off[f + 1] - prob->res_off[f]);
  lorb::InPack in(ctx);
  const int i_roff = in.add_t(prob->res_off, (size_t)nf + 1), i_intr = in.add_t(prob->intr, (size_t)nf * 4),
            i_pinit = in.add_t(prob->pose_init, (size_t)nf * 6), i_pts = in.add_t(prob->pts3d, (size_t)nr * 3),
            i_obs = in.add_t(prob->obs2d, (size_t)nr * 2);
  LORB_TRY(in.commit(max_res <= kPoRegRes));
  lorb::OutPack out(ctx);
  const int o_pose = out.add(sizeof(double) * 6 * nf), o_sum = out.add(sizeof(lorb_ba_summary) * nf);
  LORB_TRY(out.alloc(true));  // the kernel stores poses and summaries into the mapped block
  PoOff aoff{};
  if (nf <= kPoArgF) {
    aoff.n = nf;
    for (int f = 0; f <= nf; ++f) aoff.off[f] = prob->res_off[f];
  }
  hipLaunchKernelGGL(k_ba_pose_only, dim3(nf), dim3(kPoThreads), 0, ctx->stream, aoff, in.dev<int32_t>(i_roff), in.dev<float>(i_intr),
                     in.dev<float>(i_pinit), in.dev<float>(i_pts), in.dev<float>(i_obs), to_dev_opt(opt),
                     out.dev<double>(o_pose), out.dev<lorb_ba_summary>(o_sum));
  LORB_CHECK_LAUNCH(ctx);
  LORB_TRY(out.fetch());
  memcpy(pose_out, out.host<double>(o_pose), sizeof(double) * 6 * nf);
  if (summaries) memcpy(summaries, out.host<lorb_ba_summary>(o_sum), sizeof(lorb_ba_summary) * nf);
  if (Tcw_out)
    for (int f = 0; f < nf; ++f) {
      const float R[3] = {(float)pose_out[6 * f], (float)pose_out[6 * f + 1], (float)pose_out[6 * f + 2]};
      const float T[3] = {(float)pose_out[6 * f + 3], (float)pose_out[6 * f + 4], (float)pose_out[6 * f + 5]};
      lorb_pose_to_Tcw(R, T, Tcw_out + 16 * f);
    }
  return LORB_OK;
}

#ifdef LORB_PO_STAMPS
int lorb_debug_po_stamps(unsigned long long* out64) {
  return hipMemcpyFromSymbol(out64, HIP_SYMBOL(g_po_st), sizeof(unsigned long long) * 64) == hipSuccess ? 0 : -1;
}
#endif

// cv::Rodrigues (vector -> matrix, double internally) + Frame::UpdatePoseMat write-back
// (the file-scope contraction pragma must not reach this restatement: it rounds like the
// reference's un-contracted host build whatever -march the library is built with)
void lorb_pose_to_Tcw(const float rvec[3], const float tvec[3], float T[16]) {
#pragma clang fp contract(off)
  double rx = rvec[0], ry = rvec[1], rz = rvec[2];
  const double theta = std::sqrt(rx * rx + ry * ry + rz * rz);
  double R[9];
  if (theta < 2.220446049250313e-16) {
    for (int k = 0; k < 9; ++k) R[k] = (k % 4 == 0) ? 1.0 : 0.0;
  } else {
    const double c = std::cos(theta), s = std::sin(theta), c1 = 1. - c;
    const double it = theta ? 1. / theta : 0.;
    rx *= it; ry *= it; rz *= it;
    const double rrt[9] = {rx * rx, rx * ry, rx * rz, rx * ry, ry * ry, ry * rz, rx * rz, ry * rz, rz * rz};
    const double rxm[9] = {0, -rz, ry, rz, 0, -rx, -ry, rx, 0};
    const double I[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    for (int k = 0; k < 9; ++k) R[k] = c * I[k] + c1 * rrt[k] + s * rxm[k];
  }
  for (int r = 0; r < 3; ++r) {
    for (int c = 0; c < 3; ++c) T[4 * r + c] = (float)R[3 * r + c];
    T[4 * r + 3] = tvec[r];
  }
  T[12] = 0.f; T[13] = 0.f; T[14] = 0.f; T[15] = 1.f;
}

}  // extern "C"
