// ttrl_mi355x.hip — gfx950 kernels + C ABI for the batched straight-highway simulator.
//
// Hot path: AbstractEnv._simulate (abstract.py:252-282) = frames x {Road.act, Road.step}
// (road.py:461-478) over thousands of independent envs.  One workgroup owns NS vehicle
// slots of an env (NS in {32, 64, 128, 256}; two envs share a wave64 when NS = 32), one
// lane per vehicle; the state of every vehicle lives in VGPRs for the whole fused launch,
// and the per-frame "road view" (positions, headings, speeds, lane projections) is staged
// in LDS where neighbour scans, the lane-change abort sweep and the collision sweep read it
// as broadcasts.  Leader/follower searches are min/max scans over LDS tiles; the
// sequential list-order semantics of Road.act (behavior.py:229-244) are resolved with
// wavefront ballots in index order.  No MFMA: the path is gather + compare + elementwise.
//
// Numerics follow the reference float64 expression by expression (compiled with
// -ffp-contract=off); T = double is the parity path, T = float the fast path.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>

#include "ttrl_mi355x.h"
#include "ttrl_math.h"

namespace {

// Transcendentals.  The float64 ocml expansions (Payne-Hanek reduction, extra-precision
// log/exp) are register-hungry; inlined at every call site they force spills of the
// resident vehicle state.  Out of line, the fused kernel fits its register budget with no
// scratch; the call overhead is paid ~10 times per vehicle-frame.
#define TTRL_TRANSC __noinline__
__device__ TTRL_TRANSC double t_sin(double x) { return ::sin(x); }
__device__ TTRL_TRANSC double t_cos(double x) { return ::cos(x); }
__device__ TTRL_TRANSC double t_tan(double x) { return ::tan(x); }
__device__ TTRL_TRANSC double t_atan(double x) { return ::atan(x); }
__device__ TTRL_TRANSC double t_asin(double x) { return ::asin(x); }
// pow(x, y) for x >= 0, y > 0 (IDM's (v / v0)^DELTA): exp(y log x) is within ~|y log x| ulp of
// the correctly rounded power (far inside the stated tolerances) at half of ocml pow's cost.
__device__ TTRL_TRANSC double t_pow(double x, double y) { return ::exp(y * ::log(x)); }
template <typename T> struct SinCos { T s, c; };
// one shared argument reduction; ocml's sincos returns the same values as sin and cos
__device__ TTRL_TRANSC SinCos<double> t_sincos(double x) {
  SinCos<double> r;
  ::sincos(x, &r.s, &r.c);
  return r;
}
#define TTRL_TRANSC32 __forceinline__
__device__ TTRL_TRANSC32 float t_sin(float x) { return ::sinf(x); }
__device__ TTRL_TRANSC32 float t_cos(float x) { return ::cosf(x); }
__device__ TTRL_TRANSC32 float t_tan(float x) { return ::tanf(x); }
__device__ TTRL_TRANSC32 float t_atan(float x) { return ::atanf(x); }
__device__ TTRL_TRANSC32 float t_asin(float x) { return ::asinf(x); }
__device__ TTRL_TRANSC32 float t_pow(float x, float y) { return ::powf(x, y); }
__device__ TTRL_TRANSC32 SinCos<float> t_sincos(float x) {
  SinCos<float> r;
  ::sincosf(x, &r.s, &r.c);
  return r;
}

// Elementary functions of the simulate kernel's vehicle model (steering, bicycle model, IDM):
// float64 through the short inline fdlibm restatements of ttrl_math.h, float32 through ocml.
__device__ __forceinline__ SinCos<double> k_sincos(double x) {
  SinCos<double> r;
  ttrl_math::sincos_d(x, r.s, r.c);
  return r;
}
__device__ __forceinline__ double k_atan(double x) { return ttrl_math::atan_d(x); }
__device__ __forceinline__ double k_asin(double x) { return ttrl_math::asin_d(x); }
__device__ __forceinline__ double k_pow(double x, double y) { return ttrl_math::pow_d(x, y); }
__device__ __forceinline__ SinCos<float> k_sincos(float x) { return t_sincos(x); }
__device__ __forceinline__ float k_atan(float x) { return t_atan(x); }
__device__ __forceinline__ float k_asin(float x) { return t_asin(x); }
__device__ __forceinline__ float k_pow(float x, float y) { return t_pow(x, y); }

constexpr int LMAX = TTRL_MAX_LANES;
// Lanes the straight-road instance's LDS layout is sized for; a road with more lanes runs the
// NET_CURVED instance (which handles straight lanes too, with a layout sized at run time).
constexpr int STRAIGHT_LANE_CAP = 4;

// Lane exchange inside 8-lane groups on the DPP network (a VALU move, a few cycles) instead of
// ds_bpermute (an LDS round trip): K = 1 and 2 swap with lane g ^ K (quad_perm), K = 4 pairs lane
// g with 7 - g (row_half_mirror), joining the group's two quads -- all the symmetric (commutative,
// associative) group reductions below need.  Every lane of a group must be active.
template <int K> __device__ __forceinline__ int grp8_swap(int v) {
  static_assert(K == 1 || K == 2 || K == 4, "8-lane group exchange");
  return __builtin_amdgcn_mov_dpp(v, K == 1 ? 0xB1 : (K == 2 ? 0x4E : 0x141), 0xf, 0xf, false);
}
template <int K> __device__ __forceinline__ double grp8_swap(double v) {
  const int lo = grp8_swap<K>(__double2loint(v)), hi = grp8_swap<K>(__double2hiint(v));
  return __hiloint2double(hi, lo);
}
template <int K> __device__ __forceinline__ float grp8_swap(float v) {
  return __int_as_float(grp8_swap<K>(__float_as_int(v)));
}
constexpr float FAR = 1e30f;  // x of absent slots in the LDS view: never within a collision window

template <typename T> struct K;
template <> struct K<double> {
  static __device__ __forceinline__ double nan() { return __builtin_nan(""); }
  static __device__ __forceinline__ double inf() { return __builtin_inf(); }
};
template <> struct K<float> {
  static __device__ __forceinline__ float nan() { return __builtin_nanf(""); }
  static __device__ __forceinline__ float inf() { return __builtin_inff(); }
};

template <typename T> __device__ __forceinline__ T Tpi() { return T(3.141592653589793); }

// utils.py:48-54
template <typename T> __device__ __forceinline__ T not_zero(T x) {
  const T eps = T(1e-2);
  if (fabs(x) > eps) return x;
  return x >= T(0) ? eps : -eps;
}
// numpy float remainder (result has the divisor's sign)
template <typename T> __device__ __forceinline__ T pymod(T a, T b) {
  // One period either side needs no generic fmod: fmod(a, b) is a for 0 <= a < b, a - b for
  // b <= a < 2b (exact by Sterbenz, as fmod's result is), and a for -b < a < 0, which numpy then
  // moves into the divisor's sign with one rounded a + b.
  if (b > T(0)) {
    if (a >= T(0) && a < b) return a;
    if (a >= b && a < T(2) * b) return a - b;
    if (a < T(0) && a > -b) return a + b;
  }
  T m = fmod(a, b);
  if (m != T(0)) { if ((b < T(0)) != (m < T(0))) m += b; }
  else m = copysign(T(0), b);
  return m;
}
// utils.py:57-58
template <typename T> __device__ __forceinline__ T wrap_to_pi(T x) {
  return pymod(x + Tpi<T>(), T(2) * Tpi<T>()) - Tpi<T>();
}
template <typename T> __device__ __forceinline__ T clip(T x, T lo, T hi) { return x < lo ? lo : (x > hi ? hi : x); }
template <typename T> __device__ __forceinline__ T lmap(T v, T x0, T x1, T y0, T y1) {
  return y0 + (v - x0) * (y1 - y0) / (x1 - x0);  // utils.py:29-31
}

// Lane table staged in LDS as T: StraightLane lane.py:159-213, SineLane :235-290,
// CircularLane :293-350 (type: TTRL_LANE_*; a uniform branch on a straight-only road).
template <typename T> struct LaneT {
  T sx, sy, dx, dy, len, w, hd, lim;
  T amp, puls, ph;                  // SineLane
  T cx, cy, rad, sph, dirn;         // CircularLane
  int forb, type;
  int road, lid, rfirst, rn, prio;  // network: road, id within it, the road's first lane and lane count
};

// The behaviour constants as the float32 kernels use them: ttrl_params_t rounded once on the host,
// so the launch's kernel arguments are float32 and every use reads a scalar register.  Converted
// inside the kernel, the constants were hoisted out of the frame loop as VGPRs and spilled (the
// float32 straight instance's scratch segment, written back to HBM every launch).  Same values as
// T(P.x) in the kernel: float(double) rounds to nearest on the host as on the device.
struct ParamsF {
  float acc_max, comfort_acc_max, comfort_acc_min, distance_wanted, time_wanted, gap_denom, politeness,
      lane_change_min_acc_gain, lane_change_max_braking, lane_change_delay, tau_pursuit, kp_a, kp_heading, kp_lateral,
      max_steering, length, width, diagonal, max_speed, min_speed, lane_vehicle_length;
  float target_speeds[8];
  int32_t n_target_speeds;
};
template <typename T> struct ParamsSel { using type = ttrl_params_t; };
template <> struct ParamsSel<float> { using type = ParamsF; };
template <typename T> using ParamsT = typename ParamsSel<T>::type;
inline ParamsF params_f(const ttrl_params_t& p) {
  ParamsF f{};
  f.acc_max = (float)p.acc_max; f.comfort_acc_max = (float)p.comfort_acc_max; f.comfort_acc_min = (float)p.comfort_acc_min;
  f.distance_wanted = (float)p.distance_wanted; f.time_wanted = (float)p.time_wanted; f.gap_denom = (float)p.gap_denom;
  f.politeness = (float)p.politeness; f.lane_change_min_acc_gain = (float)p.lane_change_min_acc_gain;
  f.lane_change_max_braking = (float)p.lane_change_max_braking; f.lane_change_delay = (float)p.lane_change_delay;
  f.tau_pursuit = (float)p.tau_pursuit; f.kp_a = (float)p.kp_a; f.kp_heading = (float)p.kp_heading;
  f.kp_lateral = (float)p.kp_lateral; f.max_steering = (float)p.max_steering; f.length = (float)p.length;
  f.width = (float)p.width; f.diagonal = (float)p.diagonal; f.max_speed = (float)p.max_speed;
  f.min_speed = (float)p.min_speed; f.lane_vehicle_length = (float)p.lane_vehicle_length;
  for (int k = 0; k < 8; ++k) f.target_speeds[k] = (float)p.target_speeds[k];
  f.n_target_speeds = p.n_target_speeds;
  return f;
}
template <typename T> inline ParamsT<T> params_for(const ttrl_params_t& p);
template <> inline ttrl_params_t params_for<double>(const ttrl_params_t& p) { return p; }
template <> inline ParamsF params_for<float>(const ttrl_params_t& p) { return params_f(p); }

// Scalar arguments (a struct argument would be materialised in scratch); compiled out of the
// straight-road instance, so the curved lanes' trigonometry stays off its register budget.
template <typename T> struct Pair { T a, b; };
// Inlined: the curved-lane geometry runs only in the NET_CURVED / NET_GRAPH instances, where
// the call overhead cost more than the registers (intersection f64 launch 1.84 -> 1.60 ms).
#define TTRL_CURVED_ATTR __forceinline__
template <typename T>
__device__ TTRL_CURVED_ATTR Pair<T> curved_local(int type, T px, T py, T sx, T sy, T ux, T uy, T amp, T puls, T ph,
                                             T cx, T cy, T rad, T sph, T dirn) {
  Pair<T> o;
  if (type == TTRL_LANE_SINE) {  // SineLane.local_coordinates lane.py:275-279
    const T dx = px - sx, dy = py - sy;
    o.a = dx * ux + dy * uy;
    o.b = dx * (-uy) + dy * ux - amp * k_sincos(puls * o.a + ph).s;
  } else {  // CircularLane.local_coordinates lane.py:327-334
    const T dx = px - cx, dy = py - cy;
    T phi = atan2(dy, dx);
    phi = sph + wrap_to_pi(phi - sph);
    const T rr = sqrt(dx * dx + dy * dy);
    o.a = dirn * (phi - sph) * rad;
    o.b = dirn * (rad - rr);
  }
  return o;
}

// CV = false: the caller's road is the straight highway (the NET_STRAIGHT simulate instance, which
// the launcher picks only when every lane is a StraightLane along +x, direction exactly (1, 0), as
// RoadNetwork.straight_road_network builds them), so the curved call sites -- and the registers
// they pin -- are compiled out, and local_coordinates reduces to two subtractions:
// s = dx * 1 + dy * 0 = dx and r = dx * -0 + dy * 1 = dy, the same values up to the sign of a zero.
template <bool CV = true, typename T>
__device__ __forceinline__ void lane_local(const LaneT<T>& L, T px, T py, T& s, T& r) {
  if (!CV) {
    s = px - L.sx;
    r = py - L.sy;
  } else if (L.type == TTRL_LANE_STRAIGHT) {  // StraightLane.local_coordinates lane.py:209-213
    T dx = px - L.sx, dy = py - L.sy;
    s = dx * L.dx + dy * L.dy;
    r = dx * (-L.dy) + dy * L.dx;
  } else {
    const Pair<T> o = curved_local(L.type, px, py, L.sx, L.sy, L.dx, L.dy, L.amp, L.puls, L.ph, L.cx, L.cy, L.rad,
                                   L.sph, L.dirn);
    s = o.a;
    r = o.b;
  }
}

template <typename T>
__device__ TTRL_CURVED_ATTR T curved_heading(int type, T s, T hd, T amp, T puls, T ph, T rad, T sph, T dirn) {
  if (type == TTRL_LANE_SINE)  // SineLane.heading_at lane.py:269-273
    return hd + k_atan(amp * puls * k_sincos(puls * s + ph).c);
  const T phi = dirn * s / rad + sph;  // CircularLane.heading_at lane.py:318-321
  return phi + Tpi<T>() / T(2) * dirn;
}

template <bool CV = true, typename T>
__device__ __forceinline__ T heading_at(const LaneT<T>& L, T s) {
  return !CV || L.type == TTRL_LANE_STRAIGHT ? L.hd : curved_heading(L.type, s, L.hd, L.amp, L.puls, L.ph, L.rad, L.sph, L.dirn);
}

// AbstractLane.position for every lane class (lane.py:199-204, :263-267, :313-316)
template <typename T>
__device__ __forceinline__ void lane_position(const LaneT<T>& L, T s, T r, T& x, T& y) {
  if (L.type == TTRL_LANE_CIRCULAR) {
    const T phi = L.dirn * s / L.rad + L.sph;
    const T k = L.rad - r * L.dirn;
    const SinCos<T> sc = k_sincos(phi);
    x = L.cx + k * sc.c;
    y = L.cy + k * sc.s;
    return;
  }
  if (L.type == TTRL_LANE_SINE) r = r + L.amp * k_sincos(L.puls * s + L.ph).s;
  x = L.sx + s * L.dx + r * (-L.dy);
  y = L.sy + s * L.dy + r * L.dx;
}
template <typename T>
__device__ __forceinline__ void lane_position_straight(const LaneT<T>& L, T s, T r, T& x, T& y) {
  x = L.sx + s * L.dx + r * (-L.dy);  // StraightLane.position lane.py:199-204
  y = L.sy + s * L.dy + r * L.dx;
}

template <typename T>
__host__ __device__ inline LaneT<T> make_lane(const ttrl_lane_table_t& R, int l) {
  LaneT<T> L;
  L.sx = T(R.start_x[l]); L.sy = T(R.start_y[l]); L.dx = T(R.dir_x[l]); L.dy = T(R.dir_y[l]);
  L.len = T(R.length[l]); L.w = T(R.width[l]); L.hd = T(R.heading[l]); L.lim = T(R.speed_limit[l]);
  L.amp = T(R.amplitude[l]); L.puls = T(R.pulsation[l]); L.ph = T(R.phase[l]);
  L.cx = T(R.center_x[l]); L.cy = T(R.center_y[l]); L.rad = T(R.radius[l]); L.sph = T(R.start_phase[l]);
  L.dirn = T(R.direction[l]);
  L.forb = R.forbidden[l]; L.type = R.type[l];
  L.road = R.road[l]; L.lid = R.lane_id[l]; L.rfirst = R.road_first[R.road[l]]; L.rn = R.road_n[R.road[l]];
  L.prio = R.priority[l];
  return L;
}

// The bounding box of a lane's centre line, in float32 rounded outwards (a margin of 1e-3 m +
// 1e-6 of the coordinates): straight lanes their two ends, circular lanes their two ends and the
// cardinal points the arc passes; a sine lane gets no box (+-inf: never pruned).  A lower bound of
// distance_with_heading for project_items' pruning.
template <typename T>
__device__ __forceinline__ float4 lane_box(const LaneT<T>& L) {
  T x0, y0, x1, y1;
  if (L.type == TTRL_LANE_STRAIGHT) {
    const T ex = L.sx + L.len * L.dx, ey = L.sy + L.len * L.dy;
    x0 = fmin(L.sx, ex); x1 = fmax(L.sx, ex);
    y0 = fmin(L.sy, ey); y1 = fmax(L.sy, ey);
  } else if (L.type == TTRL_LANE_CIRCULAR) {
    const T a0 = L.sph, a1 = a0 + L.dirn * L.len / L.rad;
    const T lo = fmin(a0, a1), hi = fmax(a0, a1);
    // a degenerate arc (radius 0, a non-finite angle) gets no box; one sweeping a full turn or more
    // the whole circle -- so the cardinal-point walk below takes at most four steps
    if (!(isfinite(lo) && isfinite(hi) && isfinite(L.rad))) return make_float4(-INFINITY, -INFINITY, INFINITY, INFINITY);
    if (hi - lo >= T(6.283185307179586)) {
      const T r = fabs(L.rad);
      x0 = L.cx - r; x1 = L.cx + r; y0 = L.cy - r; y1 = L.cy + r;
      const float m = 1e-3f + 1e-6f * (float)(fabs(x0) + fabs(x1) + fabs(y0) + fabs(y1));
      return make_float4((float)x0 - m, (float)y0 - m, (float)x1 + m, (float)y1 + m);
    }
    x0 = x1 = L.cx + L.rad * cos(a0);
    y0 = y1 = L.cy + L.rad * sin(a0);
    const T ex = L.cx + L.rad * cos(a1), ey = L.cy + L.rad * sin(a1);
    x0 = fmin(x0, ex); x1 = fmax(x1, ex); y0 = fmin(y0, ey); y1 = fmax(y1, ey);
    const T q = T(1.5707963267948966);
    T a = ceil(lo / q) * q;
    for (int k = 0; k < 5 && a <= hi; ++k, a += q) {  // cardinal points within the arc (< 2 pi: at most 4)
      const T px = L.cx + L.rad * cos(a), py = L.cy + L.rad * sin(a);
      x0 = fmin(x0, px); x1 = fmax(x1, px); y0 = fmin(y0, py); y1 = fmax(y1, py);
    }
  } else {
    return make_float4(-INFINITY, -INFINITY, INFINITY, INFINITY);
  }
  const float m = 1e-3f + 1e-6f * (float)(fabs(x0) + fabs(x1) + fabs(y0) + fabs(y1));
  return make_float4((float)x0 - m, (float)y0 - m, (float)x1 + m, (float)y1 + m);
}

// AbstractLane.is_reachable_from lane.py:104-118
template <bool CV = true, typename T>
__device__ __forceinline__ bool reachable(const LaneT<T>& L, T vl, T px, T py) {
  if (L.forb) return false;
  T s, r;
  lane_local<CV>(L, px, py, s, r);
  return fabs(r) <= T(2) * L.w && T(0) <= s && s < L.len + vl;
}

// ControlledVehicle.steering_control controller.py:145-187, from the vehicle's local coordinates
// (s, r) on its target lane L
template <bool CV = true, typename T, typename PP>
__device__ __forceinline__ T steering_control_sr(const LaneT<T>& L, const PP& P, T s, T r, T h, T v) {
  const T lfh = heading_at<CV>(L, s + v * T(P.tau_pursuit));  // lane_future_heading
  const T lat_cmd = -T(P.kp_lateral) * r;
  const T hcmd = k_asin(clip(lat_cmd / not_zero(v), T(-1), T(1)));
  const T href = lfh + clip(hcmd, -Tpi<T>() / T(4), Tpi<T>() / T(4));
  const T hrate = T(P.kp_heading) * wrap_to_pi(href - h);
  // slip = asin(c); tan(slip) = c / sqrt((1 - c)(1 + c)) (= +-inf at |c| = 1, where the
  // reference's tan(+-pi/2) = +-1.6e16 and atan of either is +-pi/2): one call instead of two
  const T c = clip(T(P.length) / T(2) / not_zero(v) * hrate, T(-1), T(1));
  const T st = k_atan(T(2) * (c / sqrt((T(1) - c) * (T(1) + c))));
  return clip(st, -T(P.max_steering), T(P.max_steering));
}
template <bool CV = true, typename T, typename PP>
__device__ __forceinline__ T steering_control(const LaneT<T>& L, const PP& P, T x, T y, T h, T v) {
  T s, r;
  lane_local<CV>(L, x, y, s, r);
  return steering_control_sr<CV>(L, P, s, r, h, v);
}

// MDPVehicle.speed_to_index controller.py:326-344 (np.round: half to even)
template <typename T, typename PP>
__device__ __forceinline__ int speed_to_index(const PP& P, T v) {
  const int n = P.n_target_speeds;
  const T x = (v - T(P.target_speeds[0])) / (T(P.target_speeds[n - 1]) - T(P.target_speeds[0]));
  return (int)clip(rint(x * T(n - 1)), T(0), T(n - 1));
}

#ifndef TTRL_SIM_WAVES
#define TTRL_SIM_WAVES 0   // min waves/SIMD for the fused kernel; 0 = tuned default (f64: 2, f32: 4)
#endif
#define TTRL_SAT_ATTR

// utils.are_polygons_intersecting utils.py:194-239 on the closed 5-point rectangles of
// RoadObject.polygon objects.py:168-180.  a = lower-index vehicle (the reference's self).
template <typename T, typename PP>
__device__ TTRL_SAT_ATTR void sat_pair(const PP& P, T ax, T ay, T ac, T as, T av, T bx, T by, T bc, T bs, T bv,
                         T dt, bool& inter, bool& will, T& tx, T& ty) {
  const T hl = T(P.length) / T(2), hw = T(P.width) / T(2);
  const T lx[4] = {-hl, -hl, +hl, +hl}, ly[4] = {-hw, +hw, +hw, -hw};
  T pa[5][2], pb[5][2];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    pa[k][0] = ac * lx[k] + (-as) * ly[k] + ax;
    pa[k][1] = as * lx[k] + ac * ly[k] + ay;
    pb[k][0] = bc * lx[k] + (-bs) * ly[k] + bx;
    pb[k][1] = bs * lx[k] + bc * ly[k] + by;
  }
  pa[4][0] = pa[0][0]; pa[4][1] = pa[0][1];
  pb[4][0] = pb[0][0]; pb[4][1] = pb[0][1];
  const T dax = av * ac * dt, day = av * as * dt, dbx = bv * bc * dt, dby = bv * bs * dt;
  const T cax = (((pa[0][0] + pa[1][0]) + pa[2][0]) + pa[3][0]) / T(4);
  const T cay = (((pa[0][1] + pa[1][1]) + pa[2][1]) + pa[3][1]) / T(4);
  const T cbx = (((pb[0][0] + pb[1][0]) + pb[2][0]) + pb[3][0]) / T(4);
  const T cby = (((pb[0][1] + pb[1][1]) + pb[2][1]) + pb[3][1]) / T(4);
  bool it = true, wi = true;
  T mind = K<T>::inf(), axx = T(0), axy = T(0);
#pragma unroll
  for (int pi = 0; pi < 2; ++pi) {
    bool brk = false;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (brk) continue;
      const T(*pg)[2] = pi == 0 ? pa : pb;
      T nx = -pg[e + 1][1] + pg[e][1], ny = pg[e + 1][0] - pg[e][0];
      const T nn = sqrt(nx * nx + ny * ny);
      nx /= nn; ny /= nn;
      T mina = T(0), maxa = T(0), minb = T(0), maxb = T(0);
#pragma unroll
      for (int k = 0; k < 5; ++k) {
        const T p = pa[k][0] * nx + pa[k][1] * ny;
        if (k == 0 || p < mina) mina = p;
        if (k == 0 || p > maxa) maxa = p;
        const T q = pb[k][0] * nx + pb[k][1] * ny;
        if (k == 0 || q < minb) minb = q;
        if (k == 0 || q > maxb) maxb = q;
      }
      if ((mina < minb ? minb - maxa : mina - maxb) > T(0)) it = false;
      const T vp = nx * (dax - dbx) + ny * (day - dby);
      if (vp < T(0)) mina += vp; else maxa += vp;
      const T dist = mina < minb ? minb - maxa : mina - maxb;
      if (dist > T(0)) wi = false;
      if (!it && !wi) { brk = true; continue; }
      if (fabs(dist) < mind) {
        mind = fabs(dist);
        const T dx = cax - cbx, dy = cay - cby;
        if (dx * nx + dy * ny > T(0)) { axx = nx; axy = ny; } else { axx = -nx; axy = -ny; }
      }
    }
  }
  inter = it; will = wi;
  tx = wi ? mind * axx : T(0);
  ty = wi ? mind * axy : T(0);
}

// Conservative proof that sat_pair returns (false, false): some edge normal of either
// rectangle separates a, swept by its relative displacement, from b by more than a margin
// that dominates the rounding of the reference's corner/normal/projection arithmetic.
// The 8 normals are +-u and +-w of each box (u = heading, w = its left normal); on axis n a
// box projects to centre.n +- (hl |u.n| + hw |w.n|), and the sweep widens a's interval by
// |D.n| at most.  Pairs it cannot separate go to the exact sat_pair.
template <typename T> struct SepTol;
template <> struct SepTol<double> { static constexpr double abs = 1e-6, rel = 1e-12, quad = 1e-14; };
template <> struct SepTol<float> { static constexpr float abs = 1e-3f, rel = 1e-6f, quad = 1e-7f; };
// The reference's projections run on corners and on normals rebuilt from corner differences:
// near |x| their error grows like ulp(x) * |x| / edge, hence the quadratic term.
template <typename T> __device__ __forceinline__ T sat_margin(T ax, T ay, T bx, T by) {
  const T X = fmax(fmax(fabs(ax), fabs(ay)), fmax(fabs(bx), fabs(by)));
  return T(SepTol<T>::abs) + T(SepTol<T>::rel) * X + T(SepTol<T>::quad) * X * X;
}

template <typename T, typename PP>
__device__ __forceinline__ bool sat_separated(const PP& P, T ax, T ay, T ac, T as, T av, T bx, T by, T bc,
                                              T bs, T bv, T dt) {
  const T hl = T(P.length) / T(2), hw = T(P.width) / T(2);
  const T dx = bx - ax, dy = by - ay;
  const T Dx = (av * ac - bv * bc) * dt, Dy = (av * as - bv * bs) * dt;
  const T C = fabs(ac * bc + as * bs), S = fabs(as * bc - ac * bs);
  const T ru = hl + hl * C + hw * S;  // both boxes' half extents along either box's u
  const T rw = hw + hw * C + hl * S;  // ... along either box's w
  const T m = sat_margin(ax, ay, bx, by);
  const T g1 = fabs(dx * ac + dy * as) - fabs(Dx * ac + Dy * as) - ru;
  const T g2 = fabs(dy * ac - dx * as) - fabs(Dy * ac - Dx * as) - rw;
  const T g3 = fabs(dx * bc + dy * bs) - fabs(Dx * bc + Dy * bs) - ru;
  const T g4 = fabs(dy * bc - dx * bs) - fabs(Dy * bc - Dx * bs) - rw;
  return g1 > m || g2 > m || g3 > m || g4 > m;
}

// One edge normal of sat_pair, evaluated exactly as sat_pair's loop body does (same corners,
// same normal normalisation, same projection, branch and sweep arithmetic): axis k < 4 is
// edge k of a's polygon, k >= 4 edge k-4 of b's.  Returns the static and swept interval
// distances and the normal oriented along the centre difference (the translation axis).
template <typename T, typename PP>
__device__ __forceinline__ void sat_axis(const PP& P, int k, T ax, T ay, T ac, T as, T av, T bx, T by,
                                         T bc, T bs, T bv, T dt, T& dd, T& dist, T& axx, T& axy) {
  const T hl = T(P.length) / T(2), hw = T(P.width) / T(2);
  const T lx[4] = {-hl, -hl, +hl, +hl}, ly[4] = {-hw, +hw, +hw, -hw};
  T pa[4][2], pb[4][2];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    pa[c][0] = ac * lx[c] + (-as) * ly[c] + ax;
    pa[c][1] = as * lx[c] + ac * ly[c] + ay;
    pb[c][0] = bc * lx[c] + (-bs) * ly[c] + bx;
    pb[c][1] = bs * lx[c] + bc * ly[c] + by;
  }
  const int e = k & 3, e1 = (e + 1) & 3;
  const bool own_b = k >= 4;
  // corners e and e+1 of the edge's polygon (selects, no dynamic register indexing)
  T p1x = pa[0][0], p1y = pa[0][1], p2x = pa[1][0], p2y = pa[1][1];
#pragma unroll
  for (int c = 1; c < 4; ++c) {
    if (e == c) { p1x = own_b ? pb[c][0] : pa[c][0]; p1y = own_b ? pb[c][1] : pa[c][1]; }
    if (e1 == c) { p2x = own_b ? pb[c][0] : pa[c][0]; p2y = own_b ? pb[c][1] : pa[c][1]; }
  }
  if (e == 0) { p1x = own_b ? pb[0][0] : pa[0][0]; p1y = own_b ? pb[0][1] : pa[0][1]; }
  if (e1 == 0) { p2x = own_b ? pb[0][0] : pa[0][0]; p2y = own_b ? pb[0][1] : pa[0][1]; }
  T nx = -p2y + p1y, ny = p2x - p1x;
  const T nn = sqrt(nx * nx + ny * ny);
  nx /= nn; ny /= nn;
  T mina = T(0), maxa = T(0), minb = T(0), maxb = T(0);
#pragma unroll
  for (int c = 0; c < 4; ++c) {  // the closing 5th point repeats corner 0: same min / max
    const T p = pa[c][0] * nx + pa[c][1] * ny;
    if (c == 0 || p < mina) mina = p;
    if (c == 0 || p > maxa) maxa = p;
    const T q = pb[c][0] * nx + pb[c][1] * ny;
    if (c == 0 || q < minb) minb = q;
    if (c == 0 || q > maxb) maxb = q;
  }
  dd = mina < minb ? minb - maxa : mina - maxb;
  const T dax = av * ac * dt, day = av * as * dt, dbx = bv * bc * dt, dby = bv * bs * dt;
  const T vp = nx * (dax - dbx) + ny * (day - dby);
  if (vp < T(0)) mina += vp; else maxa += vp;
  dist = mina < minb ? minb - maxa : mina - maxb;
  const T cax = (((pa[0][0] + pa[1][0]) + pa[2][0]) + pa[3][0]) / T(4);
  const T cay = (((pa[0][1] + pa[1][1]) + pa[2][1]) + pa[3][1]) / T(4);
  const T cbx = (((pb[0][0] + pb[1][0]) + pb[2][0]) + pb[3][0]) / T(4);
  const T cby = (((pb[0][1] + pb[1][1]) + pb[2][1]) + pb[3][1]) / T(4);
  const T dx = cax - cbx, dy = cay - cby;
  if (dx * nx + dy * ny > T(0)) { axx = nx; axy = ny; } else { axx = -nx; axy = -ny; }
}

// sat_pair for the rare overflow sweep, its results returned by value: the compiler keeps this
// call out of line in the register-heavy road-network instance, and out-parameters of a call
// would live in scratch.  flags: bit 0 intersecting, bit 1 will_intersect.
template <typename T> struct SatRes { T tx, ty; int flags; };
template <typename T, typename PP>
__device__ SatRes<T> sat_pair_v(const PP& P, T ax, T ay, T ac, T as, T av, T bx, T by, T bc, T bs, T bv, T dt) {
  bool inter, will;
  SatRes<T> o;
  sat_pair(P, ax, ay, ac, as, av, bx, by, bc, bs, bv, dt, inter, will, o.tx, o.ty);
  o.flags = (inter ? 1 : 0) | (will ? 2 : 0);
  return o;
}

// ---------------------------------------------------------------------------------
// Per-lane candidate lists: for every lane, the longitudinal coordinates of the env's
// vehicles that are on it (keys) and their slots (idx), in slot order; each vehicle also
// records its own position in the lists it belongs to (mypos, -1 if not on the lane).

// Road topology of the network (ttrl_lane_table_t road_*), staged in LDS for the route helpers.
struct RoadTab {
  int from[TTRL_MAX_ROADS], to[TTRL_MAX_ROADS], first[TTRL_MAX_ROADS], n[TTRL_MAX_ROADS];
  int n_roads;
};

// The collision queue holds close pairs (i < j) for the SAT test as three arrays: the translation
// (tx, ty) and ij = i | j << 8 | result << 16 (bit 0 intersecting, bit 1 will_intersect).
__device__ __forceinline__ int pair_pack(int i, int j, int res) { return i | (j << 8) | (res << 16); }

// LDS "road view" of one workgroup (EPW envs x NS slots).
template <typename T> struct View {
  LaneT<T>* lanes;   // [LMAX]
  T *x, *y, *v, *ch, *sh, *ts;  // [EPW*NS] shared road view (read by other vehicles)
  float* xf;                     // [EPW*NS] float copy of x for the collision window prefilter (== x for f32)
  T *h, *delta;                  // [EPW*NS] heading (project_items reads it across lanes), IDM DELTA (MOBIL items)
  T* afree;                      // [EPW*NS] IDM free-road term of the frame (MOBIL items read it)
  T* powb;                       // [EPW*NS] its power's base (pow_base), any vehicle's (MOBIL items)
  uint8_t *kind, *flags;         // [EPW*NS] flags: 1 crashed, 2 has_impact, 4 enable_lane_change
  T* key;            // [n_lanes][EPW][NS+1] s of the vehicles on each lane (AbstractLane.on_lane margin 1)
  uint8_t* idx;      // [n_lanes][EPW][NS+1] their slots, slot order
  short* mypos;      // [n_lanes][EPW*NS] each vehicle's position in the list, -1 if not on the lane
  short *f0, *r0, *ft;  // [EPW*NS] own-lane front / rear, target-lane front of the frame (-1 none)
  short* mob;        // [2][EPW*NS] MOBIL verdict per side: -2 refused, else the new front (-1 none)
  short* item;       // [EPW][2*NS] MOBIL work items: slot | side << 15
  int* cnt;          // [EPW][LMAX+1] list lengths; [LMAX] = longest list of the env
  int* wcnt;         // [LMAX][4] per-wave list lengths (NS > 64)
  int* nitem;        // [EPW] MOBIL items queued this frame
  int8_t *lane, *tgt;            // [EPW*NS] lane (-1 absent), target (old, for the act phase)
  unsigned long long* bal;       // [2][8] cross-wave ballots (NS > 64)
  T *pq_tx, *pq_ty;              // [EPW][NS] close vehicle pairs of the frame (collision queue) ...
  int* pq_ij;                    // ... over the act phase's scratch (afree .. item), dead by then
  int* pq_n;                     // [EPW] queue lengths (> NS: overflow)
  // NET_GRAPH only (null otherwise)
  int8_t *rroad, *rlane;         // [EPW*NS][TTRL_ROUTE_MAX] routes
  int8_t* rn;                    // [EPW*NS] route lengths (-1 None)
  uint8_t* ynew;                 // [EPW*NS] RegulatedRoad: yields decided this enforcement
  RoadTab* rt;                   // road topology
  int* rq;                       // [rq_cap] RegulatedRoad (pair, time step) items past the float prefilter,
  uint8_t* rqf;                  // [RQ_PAIRS] and the pairs' conflict flags: the dead transient block
  int rq_cap;                    // beyond the predictions (0: no room, the serial pair loop runs)
  float *px, *py;                // [EPW*NS][PRED_T] predicted positions, float32 (is_conflict_possible's
                                 // distance prefilter; poses that pass are recomputed in float64)
  T* ps0;                        // [EPW*NS] the prediction's start: s along the current lane
  unsigned long long* onm;       // [LMAX] (vehicle, lane) projection: on-lane slot masks
  uint8_t* live;                 // [EPW*NS] present slots in slot order
  int8_t* lperm;                 // [LMAX] lanes, straight ones first
  T* pd;                         // [EPW*NS] per-item-thread closest distance so far
  int8_t* pl;                    // [EPW*NS] ... and its lane (-1 none)
  // Straight instance, one wavefront (sorted_view): the env's vehicles in (x, slot) order instead
  // of the per-lane lists (key / idx / mypos are not allocated)
  uint8_t* onb;                  // [EPW*NS] lanes the vehicle is on (bit l: AbstractLane.on_lane margin 1)
  uint8_t *sord, *spos;          // [EPW*NS] slot at each sorted position / sorted position of each slot
  float* sxf;                    // [EPW*NS] xf at each sorted position (collision window walk)
  unsigned long long* lmask;     // [EPW][lanes] per lane: sorted positions of the vehicles on it
  int* stie;                     // [EPW] the order has ties in some lane's s (use the slot scans)
  T *steer, *acc, *ix, *iy;      // [EPW*NS] the action and the pending impact (only the vehicle reads them)
};
constexpr int PRED_T = 11;       // np.arange(0.25, 3, 0.25) (regulation.py:86)
// Per-lane list capacity of the one-wavefront road-network instance: key / idx rows hold the first
// GRAPH_LIST_CAP vehicles of a lane in list order (an intersection scene has ~8 live vehicles per
// env over 20 lanes); the rest of a longer list is walked from the lane's on-lane slot mask with
// its s recomputed (the same lane_local bits).  With the predictions in float32 this keeps the
// float64 view <= 20 KB: 8 workgroups per CU, a 4096-env batch in one round.
constexpr int GRAPH_LIST_CAP = 14;
// Capacity of a list row: every slot of the env on the other instances.
__host__ __device__ constexpr int list_cap(int NS, int EPW, bool graph) {
  return graph && NS * EPW == 64 ? GRAPH_LIST_CAP : NS;
}

// Byte offsets of the view's arrays in the dynamic LDS block (host: sizing; device: carve).
constexpr int N_REALS = 8;  // x, y, v, ch, sh, ts, h, delta
constexpr int RQ_PAIRS = 256;  // RegulatedRoad pairs of a wave the flattened enforcement takes (else serial)
struct ViewLayout {
  size_t lanes, reals[N_REALS], xf, key, afree, powb, pq_tx, pq_ty, pq_ij, bal, cnt, wcnt, nitem, pq_n, mypos, f0, r0, ft,
      mob, item, idx, kind, flags, lane, tgt, pred, rroad, rlane, rn, ynew, rt, onm, live, lperm, pd, pl, onb, sord,
      spos, sxf, lmask, stie, own, rq, rqf, rq_cap, total;
};

template <typename T>
__host__ __device__ inline ViewLayout view_layout(int EPW, int NS, int n_lanes, bool graph = false,
                                                  bool sorted = false) {
  ViewLayout o{};
  size_t p = 0;
  const size_t M = (size_t)EPW * NS;
  auto take = [&](size_t bytes, size_t align) {
    p = (p + align - 1) & ~(align - 1);
    const size_t r = p;
    p += bytes;
    return r;
  };
  o.lanes = take(sizeof(LaneT<T>) * n_lanes, 16);
  for (int k = 0; k < N_REALS; ++k) o.reals[k] = take(sizeof(T) * M, 16);
  o.xf = sizeof(T) == 8 ? take(sizeof(float) * M, 16) : o.reals[0];
  o.bal = take(NS > 64 ? 16 * sizeof(unsigned long long) : 0, 16);  // cross-wave ballots
  o.cnt = take(sizeof(int) * EPW * (LMAX + 1), 4);
  o.wcnt = take(NS > 64 ? sizeof(int) * LMAX * 4 : 0, 4);
  o.nitem = take(sizeof(int) * EPW, 4);
  o.pq_n = take(sizeof(int) * EPW, 4);
  o.kind = take(M, 4);
  o.flags = take(M, 4);
  o.lane = take(M, 4);
  o.tgt = take(M, 4);
  // The straight one-wave instance (4 waves per SIMD, 128 VGPRs) keeps each vehicle's action and
  // pending impact here rather than in registers: its view leaves 2.4 KB per float64 env under
  // the 10 KB budget, and as registers they were spilled to scratch (written back to HBM).
  o.own = take(sorted ? sizeof(T) * 4 * M : 0, 16);
  // Frame-transient block: the per-lane candidate lists (written by the projection at the end of
  // a frame's step, read by the next frame's act), the act phase's neighbour / MOBIL scratch (read
  // from the start of a frame's act until its last barrier) and, over that scratch, the collision
  // pair queue (written after the projection).  The RegulatedRoad trajectory predictions live only
  // between the act and the kinematics, so on a road network they share the whole block.
  const size_t t0 = take(0, 16);
  if (sorted) {  // the sorted order replaces the lists (the projection writes it, the act reads it)
    o.sxf = take(sizeof(float) * M, 16);
    o.lmask = take(sizeof(unsigned long long) * EPW * n_lanes * ((NS + 63) / 64), 8);
    o.stie = take(sizeof(int) * EPW, 4);
    o.onb = take(M, 4);
    o.sord = take(M, 4);
    o.spos = take(M, 4);
  } else {
    const size_t LS = list_cap(NS, EPW, graph) + 1;
    o.key = take(sizeof(T) * (size_t)n_lanes * EPW * LS, 16);
    o.mypos = take(sizeof(short) * (size_t)n_lanes * M, 4);
    o.idx = take((size_t)n_lanes * EPW * LS, 4);
  }
  const size_t u0 = take(0, 16);
  o.afree = take(sizeof(T) * M, 16);
  o.powb = take(sizeof(T) * M, 16);
  o.f0 = take(sizeof(short) * M, 4);
  o.r0 = take(sizeof(short) * M, 4);
  o.ft = take(sizeof(short) * M, 4);
  o.mob = take(sizeof(short) * 2 * M, 4);
  o.item = take(sizeof(short) * 2 * M, 4);
  const size_t u1 = take(0, 16);
  p = u0;
  o.pq_tx = take(sizeof(T) * M, 16);
  o.pq_ty = take(sizeof(T) * M, 16);
  o.pq_ij = take(sizeof(int) * M, 4);
  if (p < u1) p = u1;
  if (graph) {
    o.pred = t0;  // float px, py [M][PRED_T], then ps0 [M]
    const size_t pred_end = t0 + ((sizeof(float) * 2 * PRED_T * M + 15) & ~(size_t)15) + sizeof(T) * M;
    if (p < pred_end) p = pred_end;
    // beyond the predictions, the rest of the transient block is dead during the enforcement as well
    o.rqf = (pred_end + 15) & ~(size_t)15;
    o.rq = o.rqf + RQ_PAIRS;
    o.rq_cap = p > o.rq + 4 * 64 ? (p - o.rq) / 4 : 0;
    o.rroad = take(TTRL_ROUTE_MAX * M, 4);
    o.rlane = take(TTRL_ROUTE_MAX * M, 4);
    o.rn = take(M, 4);
    o.ynew = take(M, 4);
    o.rt = take(sizeof(RoadTab), 4);
    o.onm = take(sizeof(unsigned long long) * LMAX, 8);
    // a T, or project_items' float2 (y, bound) per vehicle, or the regulation's reach (float) and
    // passing-pair queue (RQ_PAIRS bytes)
    o.pd = take(8 * M > 4 * M + RQ_PAIRS ? 8 * M : 4 * M + RQ_PAIRS, 16);
    o.live = take(M, 4);
    o.lperm = take(LMAX, 4);
    o.pl = take(M, 4);
  }
  o.total = take(0, 16);
  return o;
}

// Pointer arithmetic stays on the __shared__ base, so every access is a ds_* instruction
// with a 32-bit LDS address.
template <typename T>
__device__ __forceinline__ View<T> carve(char* smem, int EPW, int NS, int n_lanes, bool graph = false,
                                         bool sorted = false) {
  const ViewLayout o = view_layout<T>(EPW, NS, n_lanes, graph, sorted);
  View<T> V;
  V.lanes = (LaneT<T>*)(smem + o.lanes);
  T** reals[N_REALS] = {&V.x, &V.y, &V.v, &V.ch, &V.sh, &V.ts, &V.h, &V.delta};
  for (int k = 0; k < N_REALS; ++k) *reals[k] = (T*)(smem + o.reals[k]);
  V.xf = (float*)(smem + o.xf);
  V.key = (T*)(smem + o.key);
  V.afree = (T*)(smem + o.afree);
  V.powb = (T*)(smem + o.powb);
  V.pq_tx = (T*)(smem + o.pq_tx);
  V.pq_ty = (T*)(smem + o.pq_ty);
  V.pq_ij = (int*)(smem + o.pq_ij);
  V.bal = (unsigned long long*)(smem + o.bal);
  V.cnt = (int*)(smem + o.cnt);
  V.wcnt = (int*)(smem + o.wcnt);
  V.nitem = (int*)(smem + o.nitem);
  V.pq_n = (int*)(smem + o.pq_n);
  V.mypos = (short*)(smem + o.mypos);
  V.f0 = (short*)(smem + o.f0);
  V.r0 = (short*)(smem + o.r0);
  V.ft = (short*)(smem + o.ft);
  V.mob = (short*)(smem + o.mob);
  V.item = (short*)(smem + o.item);
  V.idx = (uint8_t*)(smem + o.idx);
  V.kind = (uint8_t*)(smem + o.kind);
  V.flags = (uint8_t*)(smem + o.flags);
  V.lane = (int8_t*)(smem + o.lane);
  V.tgt = (int8_t*)(smem + o.tgt);
  if (graph) {
    const size_t M = (size_t)EPW * NS;
    V.px = (float*)(smem + o.pred);
    V.py = V.px + PRED_T * M;
    V.ps0 = (T*)(smem + o.pred + ((sizeof(float) * 2 * PRED_T * M + 15) & ~(size_t)15));
    V.rroad = (int8_t*)(smem + o.rroad);
    V.rlane = (int8_t*)(smem + o.rlane);
    V.rn = (int8_t*)(smem + o.rn);
    V.ynew = (uint8_t*)(smem + o.ynew);
    V.rt = (RoadTab*)(smem + o.rt);
    V.rq = (int*)(smem + o.rq);
    V.rqf = (uint8_t*)(smem + o.rqf);
    V.rq_cap = (int)o.rq_cap;
    V.onm = (unsigned long long*)(smem + o.onm);
    V.pd = (T*)(smem + o.pd);
    V.live = (uint8_t*)(smem + o.live);
    V.lperm = (int8_t*)(smem + o.lperm);
    V.pl = (int8_t*)(smem + o.pl);
  }
  if (sorted) {
    V.onb = (uint8_t*)(smem + o.onb);
    V.sord = (uint8_t*)(smem + o.sord);
    V.spos = (uint8_t*)(smem + o.spos);
    V.sxf = (float*)(smem + o.sxf);
    V.lmask = (unsigned long long*)(smem + o.lmask);
    V.stie = (int*)(smem + o.stie);
    const size_t M = (size_t)EPW * NS;
    V.steer = (T*)(smem + o.own);
    V.acc = V.steer + M;
    V.ix = V.acc + M;
    V.iy = V.ix + M;
  }
  return V;
}

size_t host_view_bytes(int dtype, int EPW, int NS, int n_lanes, bool graph = false, bool sorted = false) {
  return dtype == TTRL_F64 ? view_layout<double>(EPW, NS, n_lanes, graph, sorted).total
                           : view_layout<float>(EPW, NS, n_lanes, graph, sorted).total;
}

template <typename T>
__device__ __forceinline__ void stage_lanes(View<T>& V, const ttrl_lane_table_t& R, int tid) {
  if (tid < R.n_lanes) V.lanes[tid] = make_lane<T>(R, tid);
}

// Per-thread vehicle registers.
template <typename T> struct Veh {
  T x, y, h, v, ts, timer, delta, steer, acc, ix, iy, ch, sh;
  int lane, tgt, sidx;
  int kind;
  bool crashed, hasimp, lc;
};

template <typename T>
__device__ __forceinline__ void load_veh(Veh<T>& a, const ttrl_state_t& s, size_t k) {
  const T* X = (const T*)s.x;
  a.x = X[k];
  a.y = ((const T*)s.y)[k];
  a.h = ((const T*)s.heading)[k];
  a.v = ((const T*)s.speed)[k];
  a.ts = ((const T*)s.target_speed)[k];
  a.timer = ((const T*)s.timer)[k];
  a.delta = ((const T*)s.delta)[k];
  a.steer = ((const T*)s.steer)[k];
  a.acc = ((const T*)s.acc)[k];
  a.ix = ((const T*)s.impact_x)[k];
  a.iy = ((const T*)s.impact_y)[k];
  a.lane = s.lane[k];
  a.tgt = s.target_lane[k];
  a.sidx = s.speed_index[k];
  a.kind = s.kind[k];
  a.crashed = s.crashed[k] != 0;
  a.hasimp = s.has_impact[k] != 0;
  a.lc = s.lane_change[k] != 0;
}

// SIDX = false: the speed index is left as it is in HBM (the simulate launch writes a changed one
// where it changes it, in the meta-action)
template <bool SIDX = true, typename T>
__device__ __forceinline__ void store_veh(const Veh<T>& a, const ttrl_state_t& s, size_t k) {
  ((T*)s.x)[k] = a.x;
  ((T*)s.y)[k] = a.y;
  ((T*)s.heading)[k] = a.h;
  ((T*)s.speed)[k] = a.v;
  ((T*)s.target_speed)[k] = a.ts;
  ((T*)s.timer)[k] = a.timer;
  ((T*)s.steer)[k] = a.steer;
  ((T*)s.acc)[k] = a.acc;
  ((T*)s.impact_x)[k] = a.ix;
  ((T*)s.impact_y)[k] = a.iy;
  s.lane[k] = a.lane;
  s.target_lane[k] = a.tgt;
  if (SIDX) s.speed_index[k] = a.sidx;
  s.crashed[k] = a.crashed ? 1 : 0;
  s.has_impact[k] = a.hasimp ? 1 : 0;
}

// Lane projections of one vehicle onto every lane.  Builds, per lane, the compacted list
// of the env's vehicles that are on it (AbstractLane.on_lane margin=1, lane.py:80-102) in
// slot order (ballot + popcount prefix), so neighbour scans visit only real candidates in
// the reference's list order; returns the closest lane (RoadNetwork.get_closest_lane_index
// road.py:55-71, distance_with_heading lane.py:132-147).  All threads must call it.
// LC < NS (the one-wavefront road network): rows keep the first LC entries, and V.onm[l] gets the
// lane's on-lane mask of the whole wavefront (the rest of a longer list is walked from it).
template <typename T, int NS, int EPW, bool CV = true, bool LISTS = true, int LC = NS, typename PP>
__device__ __forceinline__ int project_all(const View<T>& V, const PP& P, int nl, int tid, int le, int i,
                                           bool present, T x, T y, T h, bool want_closest, int* onb_out = nullptr) {
  constexpr int NSP = LC + 1;
  const T vl = T(P.lane_vehicle_length);
  int best = 0, mx = 0;
  T bd = T(0), ang = T(0), prev_hd = T(0);
  int* cnt = V.cnt + le * (LMAX + 1);
  if constexpr (NS <= 64 || !LISTS) {  // !LISTS: per-thread on-lane bits, any NS
    const int sh = NS <= 64 ? (tid & 63) / NS * NS : 0;
    const unsigned long long seg = NS == 64 ? ~0ull : ((1ull << NS) - 1);
    bool have = false;  // bd / best hold a lane
    int onbits = 0;     // !LISTS: the lanes this vehicle is on
    auto lane_l = [&](int l) {
      const LaneT<T> L = V.lanes[l];
      T s, r;
      bool full = true;  // s computed (always, on a straight lane)
      if constexpr (CV) {
        if (L.type == TTRL_LANE_CIRCULAR) {
          // CircularLane.local_coordinates (lane.py:327-334) lateral part first: the atan2 of s is
          // needed only inside the on_lane band, or below the closest distance so far -- every term
          // of distance_with_heading is >= 0, so d >= |r| and a lane with |r| >= bd cannot win.
          const T dx = x - L.cx, dy = y - L.cy;
          const T rr = sqrt(dx * dx + dy * dy);
          r = L.dirn * (L.rad - rr);
          full = present && (fabs(r) <= L.w / T(2) + T(1) || (want_closest && (!have || fabs(r) < bd)));
          s = T(0);
          if (full) {
            T phi = atan2(dy, dx);
            phi = L.sph + wrap_to_pi(phi - L.sph);
            s = L.dirn * (phi - L.sph) * L.rad;
          }
        } else {
          lane_local<CV>(L, x, y, s, r);
        }
      } else {
        lane_local<CV>(L, x, y, s, r);
      }
      const bool on = full && present && fabs(r) <= L.w / T(2) + T(1) && -vl <= s && s < L.len + vl;
      if constexpr (LISTS) {
        const unsigned long long wm = __ballot(on);
        if constexpr (LC < NS) {
          if (tid == 0) V.onm[l] = wm;
        }
        const unsigned long long m = (wm >> sh) & seg;
        const int pos = on ? __popcll(m & ((1ull << i) - 1)) : -1;
        if (on && pos < LC) {
          V.key[((size_t)l * EPW + le) * NSP + pos] = s;
          V.idx[((size_t)l * EPW + le) * NSP + pos] = (uint8_t)i;
        }
        V.mypos[(size_t)l * EPW * NS + le * NS + i] = (short)pos;
        const int c = __popcll(m);
        mx = c > mx ? c : mx;
        if (i == 0) cnt[l] = c;
      } else {
        onbits |= on ? 1 << l : 0;
      }
      if (want_closest && full) {
        const T hdl = heading_at<CV>(L, s);  // distance_with_heading lane.py:132-147
        if (!have || hdl != prev_hd) ang = fabs(wrap_to_pi(h - hdl));
        prev_hd = hdl;
        T a = s - L.len; if (!(a > T(0))) a = T(0);
        T b = T(0) - s; if (!(b > T(0))) b = T(0);
        const T d = fabs(r) + a + b + T(1) * ang;
        if (!have || d < bd) { bd = d; best = l; }
        have = true;
      }
    };
    if constexpr (CV) {
      for (int l = 0; l < nl; ++l) lane_l(l);
    } else {  // the straight instance's lanes have a compile-time bound: unrolled, their projections overlap
#pragma unroll
      for (int l = 0; l < STRAIGHT_LANE_CAP; ++l)
        if (l < nl) lane_l(l);
    }
    if constexpr (!LISTS) {
      V.onb[le * NS + i] = (uint8_t)onbits;
      if (onb_out) *onb_out = onbits;
    }
  } else {
    constexpr int W = NS / 64;
    const int wave = tid >> 6, lane = tid & 63;
    for (int l = 0; l < nl; ++l) {
      const LaneT<T> L = V.lanes[l];
      T s, r;
      lane_local<CV>(L, x, y, s, r);
      const bool on = present && fabs(r) <= L.w / T(2) + T(1) && -vl <= s && s < L.len + vl;
      const unsigned long long b = __ballot(on);
      if (lane == 0) V.wcnt[l * 4 + wave] = __popcll(b);
    }
    __syncthreads();
    for (int l = 0; l < nl; ++l) {
      const LaneT<T> L = V.lanes[l];
      T s, r;
      lane_local<CV>(L, x, y, s, r);
      const bool on = present && fabs(r) <= L.w / T(2) + T(1) && -vl <= s && s < L.len + vl;
      const unsigned long long b = __ballot(on);
      int off = 0, c = 0;
#pragma unroll
      for (int w = 0; w < W; ++w) {
        const int wc = V.wcnt[l * 4 + w];
        off += w < wave ? wc : 0;
        c += wc;
      }
      const int pos = on ? off + __popcll(b & ((1ull << lane) - 1)) : -1;
      if (on) {
        V.key[(size_t)l * NSP + pos] = s;
        V.idx[(size_t)l * NSP + pos] = (uint8_t)i;
      }
      V.mypos[(size_t)l * NS + i] = (short)pos;
      mx = c > mx ? c : mx;
      if (i == 0) cnt[l] = c;
      if (want_closest) {
        const T hdl = heading_at<CV>(L, s);  // distance_with_heading lane.py:132-147
        if (l == 0 || hdl != prev_hd) ang = fabs(wrap_to_pi(h - hdl));
        prev_hd = hdl;
        T a = s - L.len; if (!(a > T(0))) a = T(0);
        T bb = T(0) - s; if (!(bb > T(0))) bb = T(0);
        const T d = fabs(r) + a + bb + T(1) * ang;
        if (l == 0 || d < bd) { bd = d; best = l; }
      }
    }
  }
  if constexpr (LISTS)
    if (i == 0) cnt[LMAX] = mx;
  return best;
}

// The env's vehicles in (x, slot) order (sorted_view instances: one wavefront, NS lanes per env).
// Sorted position p lives in lane p of the env's segment; the order of the previous frame is
// restored by odd-even transposition (vehicles pass each other rarely within a frame, so this is
// usually the check alone), a launch's first order by a bitonic sort.  my_slot (a register of the
// lane at sorted position p) carries the slot at p from frame to frame.  Results: sord / spos, the float x
// in sorted order, per lane the sorted positions of the vehicles on it, and a tie flag: when two
// present vehicles have equal s on some lane (or x is NaN) the sorted order cannot stand for the
// reference's list-order tie rules, and the callers fall back to slot-order scans.
template <typename T, int NS, int EPW>
__device__ __forceinline__ void sort_order(const View<T>& V, int nl, int tid, int le, int i, bool init, int& my_slot,
                                           T xo, int obo) {
  const int eb = le * NS;
  const int base = tid - i;  // the segment's first lane
  if (init) my_slot = i;  // a launch's first order: bitonic from slot order
  // gathered from the lane of the slot (x and lane bits are still in its registers: no barrier)
  T key = __shfl(xo, base + my_slot);
  const int ob = __shfl(obo, base + my_slot);
  const bool nan = key != key;
  if (nan) key = K<T>::inf();  // sorted last; the tie flag sends the env to the slot scans
  int pay = my_slot | ob << 8;
  auto less = [](T ka, int pa, T kb, int pb) { return ka < kb || (ka == kb && (pa & 0xff) < (pb & 0xff)); };
  auto cmpx = [&](int pt, bool valid, bool up) {  // the pair's lower lane keeps the smaller element if up
    const T pk = __shfl(key, base + pt);
    const int pp = __shfl(pay, base + pt);
    const bool pl = less(pk, pp, key, pay);
    const bool take = valid && ((i < pt) == up ? pl : !pl);
    key = take ? pk : key;
    pay = take ? pp : pay;
  };
  if (init) {
#pragma unroll
    for (int k = 2; k <= NS; k <<= 1)
#pragma unroll
      for (int j = k >> 1; j > 0; j >>= 1) cmpx(i ^ j, true, (i & k) == 0);
  }
  T nk;
  int np;
  for (int pass = 0;; ++pass) {  // the previous frame's order, restored by odd-even transposition
    nk = __shfl(key, base + (i + 1 < NS ? i + 1 : i));
    np = __shfl(pay, base + (i + 1 < NS ? i + 1 : i));
    const bool ok = i + 1 >= NS || less(key, pay, nk, np);
    if (__all(ok) || pass == NS) break;
    cmpx(i ^ 1, true, true);
    const int po = (i & 1) ? i + 1 : i - 1;
    cmpx(po >= 0 && po < NS ? po : i, po >= 0 && po < NS, true);
  }
  const int sl = pay & 0xff;
  my_slot = sl;
  V.sord[eb + i] = (uint8_t)sl;
  V.spos[eb + sl] = (uint8_t)i;
  V.sxf[eb + i] = (float)key;
  const int sh = (tid & 63) - i;
  const unsigned long long seg = NS == 64 ? ~0ull : ((1ull << NS) - 1);
#pragma unroll
  for (int l = 0; l < STRAIGHT_LANE_CAP; ++l) {
    const unsigned long long m = (__ballot((pay >> (8 + l)) & 1) >> sh) & seg;
    if (i == 0 && l < nl) V.lmask[le * STRAIGHT_LANE_CAP + l] = m;
  }
  bool tie = nan;
  if (i + 1 < NS && key < T(FAR) && nk < T(FAR)) {
    tie |= !less(key, pay, nk, np) || nk == key;  // unsorted at the pass cap (not expected) / equal x
#pragma unroll
    for (int l = 0; l < STRAIGHT_LANE_CAP; ++l)
      if (l < nl) tie |= (key - V.lanes[l].sx) == (nk - V.lanes[l].sx);
  }
  const unsigned long long tb = (__ballot(tie) >> sh) & seg;
  if (i == 0) V.stie[le] = tb != 0;
}

// sort_order for one 128-slot env over two wavefronts (NS = 128, EPW = 1): sorted position p lives
// in thread p, which carries the slot at p in my_slot.  The slots' x and on-lane bits are read
// from the view (written by the kinematics and project_all before the call); the exchanges across
// the wave boundary -- the bitonic j = 64 stage of a launch's first order, the odd-even pair
// (63, 64), the sortedness and tie checks -- go through LDS (the act phase's scratch, dead here).
template <typename T>
__device__ __forceinline__ void sort_order128(const View<T>& V, int nl, int tid, bool init, int& my_slot) {
  constexpr int NS = 128;
  T* xk = V.afree;          // [128] keys for the cross-wave exchanges
  int* xp = (int*)V.mob;    // [128] payloads
  __syncthreads();  // every slot's x and on-lane bits are in the view
  if (init) my_slot = tid;
  T key = V.x[my_slot];
  const int ob = V.onb[my_slot];
  const bool nan = key != key;
  if (nan) key = K<T>::inf();
  int pay = my_slot | ob << 8;
  const int lane = tid & 63;
  auto less = [](T ka, int pa, T kb, int pb) { return ka < kb || (ka == kb && (pa & 0xff) < (pb & 0xff)); };
  auto apply = [&](int pt, T pk, int pp, bool valid, bool up) {
    const bool pl = less(pk, pp, key, pay);
    const bool take = valid && ((tid < pt) == up ? pl : !pl);
    key = take ? pk : key;
    pay = take ? pp : pay;
  };
  if (init) {
#pragma unroll
    for (int k = 2; k <= NS; k <<= 1)
#pragma unroll
      for (int j = k >> 1; j > 0; j >>= 1) {
        if (j == 64) {
          xk[tid] = key; xp[tid] = pay;
          __syncthreads();
          const T pk = xk[tid ^ 64];
          const int pp = xp[tid ^ 64];
          __syncthreads();
          apply(tid ^ 64, pk, pp, true, (tid & k) == 0);
        } else {
          apply(tid ^ j, __shfl(key, lane ^ j), __shfl(pay, lane ^ j), true, (tid & k) == 0);
        }
      }
  }
  T nk;
  int np;
  for (int pass = 0;; ++pass) {  // the previous frame's order, restored by odd-even transposition
    if (tid == 64) { xk[0] = key; xp[0] = pay; }
    __syncthreads();
    nk = __shfl(key, lane < 63 ? lane + 1 : lane);
    np = __shfl(pay, lane < 63 ? lane + 1 : lane);
    if (tid == 63) { nk = xk[0]; np = xp[0]; }
    const bool ok = tid + 1 >= NS || less(key, pay, nk, np);
    if (__syncthreads_and(ok) || pass == NS) break;
    apply(tid ^ 1, __shfl(key, lane ^ 1), __shfl(pay, lane ^ 1), true, true);
    if (tid == 63 || tid == 64) { xk[1 + tid - 63] = key; xp[1 + tid - 63] = pay; }
    __syncthreads();
    const int po = (tid & 1) ? tid + 1 : tid - 1;
    T pk = __shfl(key, (po & 63));
    int pp = __shfl(pay, (po & 63));
    if (tid == 63) { pk = xk[2]; pp = xp[2]; }
    if (tid == 64) { pk = xk[1]; pp = xp[1]; }
    apply(po >= 0 && po < NS ? po : tid, pk, pp, po >= 0 && po < NS, true);
    __syncthreads();  // the boundary slots are rewritten by the next pass
  }
  const int sl = pay & 0xff;
  my_slot = sl;
  V.sord[tid] = (uint8_t)sl;
  V.spos[sl] = (uint8_t)tid;
  V.sxf[tid] = (float)key;
#pragma unroll
  for (int l = 0; l < STRAIGHT_LANE_CAP; ++l) {
    const unsigned long long m = __ballot((pay >> (8 + l)) & 1);
    if (lane == 0 && l < nl) V.lmask[l * 2 + (tid >> 6)] = m;
  }
  bool tie = nan;
  if (tid + 1 < NS && key < T(FAR) && nk < T(FAR)) {
    tie |= !less(key, pay, nk, np) || nk == key;  // unsorted at the pass cap (not expected) / equal x
#pragma unroll
    for (int l = 0; l < STRAIGHT_LANE_CAP; ++l)
      if (l < nl) tie |= (key - V.lanes[l].sx) == (nk - V.lanes[l].sx);
  }
  const bool any_tie = __syncthreads_or(tie);
  if (tid == 0) V.stie[0] = any_tie;
}

// Road.neighbour_vehicles (road.py:480-513) on lane l for the vehicle at sorted position p, from
// the lane's position mask (no ties: positions order the keys strictly); slots, -1 for none.
template <typename T, int NS>
__device__ __forceinline__ void sorted_nbrs(const View<T>& V, int le, int l, int p, int& f, int& r) {
  if constexpr (NS <= 64) {
    const unsigned long long m = V.lmask[le * STRAIGHT_LANE_CAP + l] & ~(1ull << p);
    const unsigned long long up = m & ~((2ull << p) - 1), dn = m & ((1ull << p) - 1);
    f = up ? (int)V.sord[le * NS + __ffsll((long long)up) - 1] : -1;
    r = dn ? (int)V.sord[le * NS + 63 - __clzll((long long)dn)] : -1;
  } else {  // 128 positions in two words (sort_order128)
    static_assert(NS == 128, "two mask words");
    const unsigned long long* w = V.lmask + (le * STRAIGHT_LANE_CAP + l) * 2;
    const int wp = p >> 6, b = p & 63;
    const unsigned long long own = w[wp] & ~(1ull << b);
    const unsigned long long up = own & ~((2ull << b) - 1), dn = own & ((1ull << b) - 1);
    int fp = -1, rp = -1;
    if (up) fp = (wp << 6) + __ffsll((long long)up) - 1;
    else if (wp == 0 && w[1]) fp = 64 + __ffsll((long long)w[1]) - 1;
    if (dn) rp = (wp << 6) + 63 - __clzll((long long)dn);
    else if (wp == 1 && w[0]) rp = 63 - __clzll((long long)w[0]);
    f = fp >= 0 ? (int)V.sord[le * NS + fp] : -1;
    r = rp >= 0 ? (int)V.sord[le * NS + rp] : -1;
  }
}

// The same in the reference's list (slot) order, for envs whose sorted order has ties: front =
// min s_v >= s (ties: later slot), rear = max s_v < s (ties: earlier slot).
template <typename T, int NS>
__device__ __forceinline__ void slot_nbrs(const View<T>& V, int le, int self, int l, T s, int& f, int& r) {
  const T sx = V.lanes[l].sx;
  T sf = K<T>::inf(), sr = -K<T>::inf();
  f = -1;
  r = -1;
  for (int j = 0; j < NS; ++j) {
    if (j == self || !((V.onb[le * NS + j] >> l) & 1)) continue;
    const T xk = V.x[le * NS + j] - sx;  // lane_local's s on a straight +x lane
    if (s <= xk && xk <= sf) { sf = xk; f = j; }
    if (xk < s && xk > sr) { sr = xk; r = j; }
  }
}

// project_all for the road-network instance (one wavefront per workgroup), over (vehicle, lane)
// items: a scene holds ~8 live vehicles in its 32 slots, so one vehicle per SIMD lane left 3/4 of
// the lanes idle through the frame's longest phase (every vehicle on all 20 lanes, atan2 on the
// turns).  The live vehicles are split across the wavefront, each group of `total` lanes taking
// every G-th lane of V.lperm (straight lanes first, so an iteration rarely mixes lane classes).
// The results equal project_all's: the on-lane lists are rebuilt per lane in slot order from the
// on-lane masks, and the closest lane is the lexicographic (d, lane) minimum -- the first minimum
// of get_closest_lane_index.  All threads must call it.
// (Round 2 noted non-finite states / hangs here for the float32 road-network instance at a 4-wave
// (128-VGPR) budget.  Not reproducible from any committed source: the commit that wrote the note,
// rebuilt at 4 waves, passes its intersection GPU tests and 40 finite steps, and so does this
// source at 4 waves with round 3's item bounds checks silent (profiles/r03/netgraph_4wave/).  The
// 2-wave budget of the road networks is a tuning choice, not a correctness one.)
// Diagnostic timing slots: 20 phases, project_items' 5 steps (PJ), the regulation's 5 steps (RG)
// and 2 event counts (RG_COUNT: enforcements past RQ_PAIRS pairs, past the item queue)
constexpr int PH_SLOTS = 32;
#ifdef TTRL_PHASE_TIMING
// their accumulators, one row per wave, in LDS (namespace scope, so the helpers reach them)
__shared__ unsigned ph_acc[4][PH_SLOTS];
#define SUB_INIT(t) unsigned long long t = __builtin_readcyclecounter();
#define SUB(t, k)                                                                                 \
  do {                                                                                            \
    const unsigned long long sub_n = __builtin_readcyclecounter();                                \
    if ((threadIdx.x & 63) == 0) ph_acc[threadIdx.x >> 6][k] += (unsigned)(sub_n - t);            \
    t = sub_n;                                                                                    \
  } while (0)
#else
#define SUB_INIT(t)
#define SUB(t, k)
#endif
#define PJ_INIT SUB_INIT(pj_t)
#define PJ(k) SUB(pj_t, 20 + (k))
#define RG_INIT SUB_INIT(rg_t)
#define RG(k) SUB(rg_t, 25 + (k))
#ifdef TTRL_PHASE_TIMING
#define RG_COUNT(k) do { if ((threadIdx.x & 63) == 0) ph_acc[threadIdx.x >> 6][30 + (k)] += 1u; } while (0)
#else
#define RG_COUNT(k)
#endif
#define TTRL_ITEMS_ATTR __forceinline__
constexpr bool PROJ_PRUNE = true;
template <typename T, int NS, int EPW, int LC, typename PP>
__device__ TTRL_ITEMS_ATTR int project_items(const View<T>& V, const PP& P, int nl, int tid, int le, int i,
                             bool present, bool want_closest, float4 my_box, float onb) {
  static_assert(NS * EPW == 64, "one wavefront per workgroup");
  PJ_INIT
  constexpr int NSP = LC + 1;
  constexpr unsigned long long SEG = NS == 64 ? ~0ull : ((1ull << NS) - 1);
  const T vl = T(P.lane_vehicle_length);
  const unsigned long long below = (1ull << tid) - 1;
  const unsigned long long live = __ballot(present);
  const int total = __popcll(live);
  if (present) V.live[__popcll(live & below)] = (uint8_t)tid;
  if (tid < nl) V.onm[tid] = 0ull;
  for (int k = tid; k < nl * EPW * NS / 2; k += 64) ((int*)V.mypos)[k] = -1;  // not on the lane
  if (tid < EPW) V.cnt[tid * (LMAX + 1) + LMAX] = 0;
  // Pruned projection (exact).  distance_with_heading d = |r| + max(s - len, 0) + max(-s, 0) +
  // |angle| is at least the Euclidean distance to the lane's centre line (radially to the line or
  // its extension, then along it to its end), so at least the distance to the line's bounding box
  // (lane_box).  An item whose box lies farther than (a) the on-lane reach (|r| <= w/2 + 1 and
  // -LENGTH <= s < len + LENGTH keep a point within w/2 + 1 + LENGTH of the line) and (b) the
  // vehicle's distance to its previous lane (an upper bound of its minimum, the same arithmetic)
  // is neither on the lane nor the closest lane nor tied with it.  (A) box tests over all (vehicle,
  // lane) items, the survivors compacted in (vehicle, lperm) order; (B) their projections spread
  // over all lanes of the wave; (C) each vehicle's first minimum over its run of survivors;
  // (D) the on-lane survivors' list entries.  A scene whose survivors exceed the queue takes the
  // unpruned passes below.  Scratch: the act block, dead here (boxes, run starts, the queue), and
  // the lists' key rows (each survivor's d and lane), dead until (D) rewrites them.
  char* pscr = (char*)V.afree;
  float4* lbox = (float4*)pscr;                     // [nl]
  short* pstart = (short*)(lbox + nl);              // [65] run start of each live vehicle
  short* psv = pstart + 66;                         // [cap] survivors: slot << 5 | lperm position
  constexpr int ACT_BYTES = EPW * NS * (2 * (int)sizeof(T) + 14);  // afree .. item (view_layout)
  const int key_bytes = nl * EPW * NSP * (int)sizeof(T);
  const int cap = min((ACT_BYTES - 16 * nl - 2 * 66) / 2, key_bytes / (1 + (int)sizeof(T))) - 1;
  T* pd_ = V.key;                                   // [cap] d of each survivor
  int8_t* pl_ = (int8_t*)(pd_ + cap);               // [cap] and its lane
  if constexpr (PROJ_PRUNE) {
    if (tid < nl) lbox[tid] = my_box;
    T ub = K<T>::inf();
    if (present && want_closest) {
      const int l0 = V.lane[tid];
      if (l0 >= 0 && l0 < nl) {
        const LaneT<T> L = V.lanes[l0];
        const T x0 = V.x[tid], y0 = V.y[tid];
        T s0, r0;
        lane_local<true>(L, x0, y0, s0, r0);
        T a = s0 - L.len; if (!(a > T(0))) a = T(0);
        T b = T(0) - s0; if (!(b > T(0))) b = T(0);
        ub = fabs(r0) + a + b + T(1) * fabs(wrap_to_pi(V.h[tid] - heading_at<true>(L, s0)));
      }
    }
    // per vehicle, once: its float32 y and the box tests' bound (float32 rounding: 1e-3 m + 1e-6 of
    // the coordinates); its float32 x is V.xf
    const float fx = (float)V.x[tid], fy = (float)V.y[tid];
    const float bound = fmaxf(onb, ub < T(3.0e38f) ? (float)ub * 1.000001f : INFINITY) + 1e-3f +
                        1e-6f * (fabsf(fx) + fabsf(fy));
    ((float2*)V.pd)[tid] = make_float2(fy, bound);
  }
  __syncthreads();
  int cl = 0;
  bool pruned = false;
  if constexpr (PROJ_PRUNE) {
    // (A) box tests, (vehicle, lperm position) items in vehicle-major order
    const int nitems = total * nl;
    const float rnl = 1.0f / (float)nl;  // k / nl as (k + 1/2) / nl in float32: exact for k < 2^16
    int nsv = 0;
    for (int k0 = 0; k0 < nitems; k0 += 64) {
      const int k = k0 + tid;
      bool keep = false;
      int q = 0, kk = 0, vv = 0;
      if (k < nitems) {
        q = (int)(((float)k + 0.5f) * rnl);
        kk = k - q * nl;
        vv = V.live[q];
        const float fx = V.xf[vv];
        const float2 yb = ((const float2*)V.pd)[vv];
        const float fy = yb.x, bound = yb.y;
        const float4 bx = lbox[V.lperm[kk]];
        const float ex = fmaxf(fmaxf(bx.x - fx, fx - bx.z), 0.0f), ey = fmaxf(fmaxf(bx.y - fy, fy - bx.w), 0.0f);
        keep = !(ex * ex + ey * ey > bound * bound);  // NaN positions are kept
      }
      const unsigned long long bal = __ballot(keep);
      const int pos = nsv + __popcll(bal & below);
      if (k < nitems && kk == 0) pstart[q] = (short)pos;  // the survivors before vehicle q's run
      if (keep && pos < cap) psv[pos] = (short)(vv << 5 | kk);
      nsv += __popcll(bal);
    }
    PJ(0);
    if (nsv <= cap) {
      pruned = true;
      if (tid == 0) pstart[total] = (short)nsv;
      __syncthreads();
      // (B) the survivors' projections.  The lane that projects survivor k also writes its list entry
      // in (D): the s of its first SREG survivors stays in registers (a turn's s costs an atan2)
      constexpr int SREG = 2;
      T sreg[SREG];
#pragma unroll
      for (int u = 0; u < SREG; ++u) sreg[u] = T(0);
      for (int k = tid, u = 0; k < nsv; k += 64, ++u) {
        const int vv = psv[k] >> 5, l = V.lperm[psv[k] & 31];
        const LaneT<T> L = V.lanes[l];
        const T x = V.x[vv], y = V.y[vv];
        T s = T(0), r;
        bool full = true;  // s computed
        if (L.type == TTRL_LANE_CIRCULAR) {
          // CircularLane.local_coordinates (lane.py:327-334, as curved_local), the lateral part first:
          // beyond the vehicle's bound (> its distance to its previous lane, >= the on-lane reach) the
          // lane is neither on-lane nor the closest (d >= |r|), and its atan2 is skipped
          const T dx = x - L.cx, dy = y - L.cy;
          const T rr = sqrt(dx * dx + dy * dy);
          r = L.dirn * (L.rad - rr);
          full = !(fabs(r) > (T)((const float2*)V.pd)[vv].y);
          if (full) {
            T phi = atan2(dy, dx);
            phi = L.sph + wrap_to_pi(phi - L.sph);
            s = L.dirn * (phi - L.sph) * L.rad;
          }
        } else {
          lane_local<true>(L, x, y, s, r);
        }
#pragma unroll
        for (int w = 0; w < SREG; ++w)
          if (u == w) sreg[w] = s;
        if (full && fabs(r) <= L.w / T(2) + T(1) && -vl <= s && s < L.len + vl)  // AbstractLane.on_lane margin 1
          atomicOr(&V.onm[l], 1ull << vv);
        if (want_closest) {  // distance_with_heading lane.py:132-147
          T a = s - L.len; if (!(a > T(0))) a = T(0);
          T b = T(0) - s; if (!(b > T(0))) b = T(0);
          pd_[k] = full ? fabs(r) + a + b + T(1) * fabs(wrap_to_pi(V.h[vv] - heading_at<true>(L, s))) : K<T>::inf();
          pl_[k] = (int8_t)l;
        }
      }
      __syncthreads();
      PJ(1);
      // (C) the first minimum of each vehicle over its run (lperm order, ties to the lower lane)
      if (want_closest && present) {
        const int q = __popcll(live & below);
        T cd = T(0);
        cl = -1;
        const int k1 = pstart[q + 1];
        for (int k = pstart[q]; k < k1; k += 4) {  // four entries' loads at a time
          int lu[4];
          T du[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int kk = min(k + u, k1 - 1);
            lu[u] = pl_[kk];
            du[u] = pd_[kk];
          }
#pragma unroll
          for (int u = 0; u < 4; ++u)
            if (k + u < k1 && (cl < 0 || du[u] < cd || (du[u] == cd && lu[u] < cl))) { cd = du[u]; cl = lu[u]; }
        }
      }
      __syncthreads();  // (C)'s reads of the key rows before (D) writes them
      PJ(2);
      // (D) each on-lane survivor's list position (slot order = list order), key and slot
      for (int k = tid, u = 0; k < nsv; k += 64, ++u) {
        const int vv = psv[k] >> 5, l = V.lperm[psv[k] & 31];
        const unsigned long long m = V.onm[l];
        if (!((m >> vv) & 1ull)) continue;
        const int e = vv / NS, sl = vv % NS;
        const int pos = __popcll((m >> (e * NS)) & SEG & ((1ull << sl) - 1));
        V.mypos[(size_t)l * EPW * NS + vv] = (short)pos;
        if (pos < LC) {
          T sq = T(0), rq;
          if (u < SREG) {
#pragma unroll
            for (int w = 0; w < SREG; ++w)
              if (u == w) sq = sreg[w];
          } else {
            lane_local<true>(V.lanes[l], V.x[vv], V.y[vv], sq, rq);
          }
          const size_t base = ((size_t)l * EPW + e) * NSP;
          V.key[base + pos] = sq;
          V.idx[base + pos] = (uint8_t)sl;
        }
      }
    }
  }
  if (!pruned) {
  const int G = total > 0 ? 64 / total : 1;  // lane groups per vehicle
  const int g = total > 0 ? tid / total : 1;
  T bd = T(0), prev_hd = T(0), ang = T(0);
  int best = -1;
  // pass 1: on-lane masks and the closest lane; the first two on-lane s of the thread's items are
  // kept for pass 2 (the others are recomputed there: lane_local gives the same bits)
  int v = 0, la = -1, lb = -1;
  T sa = T(0), sb = T(0), x = T(0), y = T(0);
  if (g < G) {
    v = V.live[tid - g * total];
    x = V.x[v]; y = V.y[v];
    const T h = V.h[v];
    for (int kk = g; kk < nl; kk += G) {
      int l = V.lperm[kk];
      const LaneT<T> L = V.lanes[l];
      T s, r;
      lane_local<true>(L, x, y, s, r);
      if (fabs(r) <= L.w / T(2) + T(1) && -vl <= s && s < L.len + vl) {  // AbstractLane.on_lane margin 1
        atomicOr(&V.onm[l], 1ull << v);
        if (la < 0) { la = l; sa = s; }
        else if (lb < 0) { lb = l; sb = s; }
      }
      if (want_closest) {
        const T hdl = heading_at<true>(L, s);  // distance_with_heading lane.py:132-147
        if (best < 0 || hdl != prev_hd) ang = fabs(wrap_to_pi(h - hdl));
        prev_hd = hdl;
        T a = s - L.len; if (!(a > T(0))) a = T(0);
        T b = T(0) - s; if (!(b > T(0))) b = T(0);
        const T d = fabs(r) + a + b + T(1) * ang;
        if (best < 0 || d < bd || (d == bd && l < best)) { bd = d; best = l; }
      }
    }
  }
  if (want_closest) { V.pd[tid] = bd; V.pl[tid] = (int8_t)best; }
  __syncthreads();
  if (want_closest && present) {  // the vehicle's groups, combined as (d, lane)
    const int q = __popcll(live & below);
    T cd = T(0);
    cl = -1;
    for (int gg = 0; gg < G; ++gg) {
      const int u = gg * total + q, lu = V.pl[u];
      if (lu < 0) continue;
      const T du = V.pd[u];
      if (cl < 0 || du < cd || (du == cd && lu < cl)) { cd = du; cl = lu; }
    }
  }
  // pass 2: each on-lane item writes its vehicle's list position (slot order = list order) and,
  // within the row's capacity, its key and slot
  if (g < G) {
    const int e = v / NS, sl = v % NS;
    for (int kk = g; kk < nl; kk += G) {
      const int l = V.lperm[kk];
      const unsigned long long m = V.onm[l];
      if (!((m >> v) & 1ull)) continue;
      const int pos = __popcll((m >> (e * NS)) & SEG & ((1ull << sl) - 1));
      V.mypos[(size_t)l * EPW * NS + v] = (short)pos;
      if (pos < LC) {
        T s = l == la ? sa : sb;
        if (l != la && l != lb) {
          T r;
          lane_local<true>(V.lanes[l], x, y, s, r);
        }
        const size_t base = ((size_t)l * EPW + e) * NSP;
        V.key[base + pos] = s;
        V.idx[base + pos] = (uint8_t)sl;
      }
    }
  }
  }  // !pruned
  PJ(3);
  // the list lengths, one (lane, env) item per thread and round: nl * EPW may exceed the wavefront
  // (the deleted 16-slot, four-envs-per-wave instance at 20 lanes had 80 items, and a single
  // `tid < nl * EPW` round left lanes 16-19 with the previous frame's counts: DESIGN §3, r05e)
  for (int t = tid; t < nl * EPW; t += 64) {
    const int l = t / EPW, e = t - l * EPW;
    const int c = __popcll((V.onm[l] >> (e * NS)) & SEG);
    V.cnt[e * (LMAX + 1) + l] = c;
    atomicMax(&V.cnt[e * (LMAX + 1) + LMAX], c);
  }
  PJ(4);
  return cl;
}

// The vehicle's longitudinal position along lane l: from the lane's candidate list when the vehicle
// is on it (the projection after the last kinematics stored exactly lane_local's s for the same
// position), else lane_local itself -- saves the turns' atan2 in the act phase.
template <typename T, int NS, int EPW, int LC = NS>
__device__ __forceinline__ T lane_s(const View<T>& V, int l, int le, int i, T x, T y) {
  const int pos = V.mypos[(size_t)l * EPW * NS + le * NS + i];
  if (pos >= 0 && pos < LC) return V.key[((size_t)l * EPW + le) * (LC + 1) + pos];
  T s, r;
  lane_local(V.lanes[l], x, y, s, r);
  return s;
}

// ------------------------------------------------------------------ road network / routes
// Network mode of the simulate kernel: one straight road (the highway), one road of curved
// lanes, or a graph of roads with routes and RegulatedRoad priorities (the intersection).
enum { NET_STRAIGHT = 0, NET_CURVED = 1, NET_GRAPH = 2 };
// The straight instance on one wavefront per workgroup keeps each env's vehicles in (x, slot) order
// (sort_order) instead of per-lane candidate lists: on lanes along +x every lane's s is x minus a
// constant, so that one order ranks the candidates of every lane.
constexpr bool sorted_view(int NS, int EPW, int NET) {
  return NET == NET_STRAIGHT && (NS * EPW == 64 || (NS == 128 && EPW == 1));
}

// AbstractLane.distance lane.py:127-130
template <typename T>
__device__ T lane_dist(const LaneT<T>& L, T px, T py) {
  T s, r;
  lane_local(L, px, py, s, r);
  T a = s - L.len; if (T(0) > a) a = T(0);
  T b = T(0) - s; if (T(0) > b) b = T(0);
  return fabs(r) + a + b;
}

// RoadNetwork.next_lane_given_next_road road.py:136-154
template <typename T>
__device__ int next_given(const LaneT<T>* lanes, const RoadTab& R, int cur_road, int id, int nroad, int nid, T px,
                          T py, T& dist) {
  if (R.n[cur_road] == R.n[nroad]) {
    if (nid < 0) nid = id;
  } else {
    T bd = T(0);
    for (int l = 0; l < R.n[nroad]; ++l) {
      const T d = lane_dist(lanes[R.first[nroad] + l], px, py);
      if (l == 0 || d < bd) { bd = d; nid = l; }
    }
  }
  dist = lane_dist(lanes[R.first[nroad] + nid], px, py);
  return nid;
}

// ControlledVehicle.follow_road controller.py:135-143 + RoadNetwork.next_lane road.py:73-134:
// at the end of the target lane, continue on the route (popping its head in place) or on the
// leaving road whose lane is closest to the projected position.  Out of line: it runs a few
// times per vehicle and route.  `rr`/`rl`/`rn`: the vehicle's route in LDS.
template <typename T>
// Inlined into the NET_GRAPH instance, the only one that calls them (measured: intersection
// launch f64 1.115 -> 1.072 ms, f32 0.579 -> 0.529 ms against out-of-line calls).
#define TTRL_NET_ATTR __forceinline__
__device__ TTRL_NET_ATTR int follow_road(const LaneT<T>* lanes, const RoadTab& R, T vl, int tgt, T x, T y, int8_t* rr,
                                        int8_t* rl, int8_t* rn, T s) {  // s: the position along lanes[tgt]
  const LaneT<T>& L = lanes[tgt];
  if (!(s > L.len - vl / T(2))) return tgt;  // AbstractLane.after_end lane.py:120-125
  const int rd = L.road, id = L.lid, to = R.to[rd];
  int nroad = -1, nid = -1;
  int n = *rn;
  if (n > 0) {
    if (rr[0] == rd) {  // route.pop(0)
      for (int q = 0; q + 1 < TTRL_ROUTE_MAX; ++q) { rr[q] = rr[q + 1]; rl[q] = rl[q + 1]; }
      rr[TTRL_ROUTE_MAX - 1] = rl[TTRL_ROUTE_MAX - 1] = -1;
      *rn = (int8_t)(--n);
    }
    if (n > 0 && R.from[rr[0]] == to) { nroad = rr[0]; nid = rl[0]; }
  }
  T px, py;
  lane_position(L, s, T(0), px, py);  // projected position
  T d;
  if (nroad < 0) {
    bool found = false;
    T bd = T(0);
    for (int q = 0; q < R.n_roads; ++q) {
      if (R.from[q] != to) continue;
      const int cand = next_given(lanes, R, rd, id, q, -1, px, py, d);
      if (!found || d < bd) { bd = d; nroad = q; nid = cand; found = true; }
    }
    if (!found) return tgt;  // KeyError: no road leaves `to`
  } else {
    nid = next_given(lanes, R, rd, id, nroad, nid, px, py, d);
  }
  return R.first[nroad] + nid;
}

// ControlledVehicle.predict_trajectory_constant_speed controller.py:228-247 through
// RoadNetwork.position_heading_along_route road.py:352-389: the pose at t = 0.25 (step + 1) s
// along the route (route None or empty: the current lane) from s0, the position along the
// current lane; the heading only when eh is given.
template <typename T>
__device__ TTRL_NET_ATTR void pose_at(const LaneT<T>* lanes, const RoadTab& R, int cur, T s0, T v, const int8_t* rr,
                                     const int8_t* rl, int rn, int step, T& ex, T& ey, T* eh) {
  const bool route = rn > 0;
  const int n = route ? rn : 1;
  const int cid = lanes[cur].lid < lanes[cur].rn ? lanes[cur].lid : 0;  // None -> the current lane id
  T L = s0 + v * (T(0.25) + T(step) * T(0.25));
  int idx = 0;
  int lane = route ? R.first[rr[0]] + (rl[0] >= 0 ? rl[0] : cid) : cur;
  while (n - idx > 1 && L > lanes[lane].len) {
    L -= lanes[lane].len;
    ++idx;
    lane = R.first[rr[idx]] + (rl[idx] >= 0 ? rl[idx] : cid);
  }
  lane_position(lanes[lane], L, T(0), ex, ey);
  if (eh) *eh = heading_at(lanes[lane], L);
}

// The predicted positions at t = 0.25 .. 2.75 s, stored in float32 for is_conflict_possible's
// distance prefilter (px / py[0 .. PRED_T)); s0 for the float64 poses recomputed where it passes.
template <typename T>
__device__ TTRL_NET_ATTR void predict_poses(const LaneT<T>* lanes, const RoadTab& R, int cur, T x, T y, T v,
                                           const int8_t* rr, const int8_t* rl, int rn, float* px, float* py, T* ps0) {
  T s0, r0;
  lane_local(lanes[cur], x, y, s0, r0);
  *ps0 = s0;
  for (int t = 0; t < PRED_T; ++t) {
    T ex, ey;
    pose_at(lanes, R, cur, s0, v, rr, rl, rn, t, ex, ey, (T*)nullptr);
    px[t] = (float)ex; py[t] = (float)ey;
  }
}

// utils.rotated_rectangles_intersect utils.py:113-123: has_corner_inside both ways over the 9
// rect_corners points (corners, centre, edge midpoints, :126-155), each tested with
// point_in_rotated_rectangle :75-91 (which rotates by +angle, as written).
template <typename T>
__device__ TTRL_NET_ATTR bool rects_intersect(T ax, T ay, T ah, T bx, T by, T bh, T l, T w) {
  const SinCos<T> ca = k_sincos(ah), cb = k_sincos(bh);
  const T hl = l / T(2), hw = w / T(2);
  const T qx[9] = {-hl, -hl, hl, hl, T(0), -hl, hl, T(0), T(0)};
  const T qy[9] = {-hw, hw, hw, -hw, T(0), T(0), T(0), -hw, hw};
  for (int side = 0; side < 2; ++side) {
    const T c1 = side ? cb.c : ca.c, s1 = side ? cb.s : ca.s, x1 = side ? bx : ax, y1 = side ? by : ay;
    const T c2 = side ? ca.c : cb.c, s2 = side ? ca.s : cb.s, x2 = side ? ax : bx, y2 = side ? ay : by;
    for (int q = 0; q < 9; ++q) {
      const T px = c1 * qx[q] + (-s1) * qy[q] + x1, py = s1 * qx[q] + c1 * qy[q] + y1;
      const T dx = px - x2, dy = py - y2;
      const T u = c2 * dx + (-s2) * dy, v = s2 * dx + c2 * dy;
      if (-l / T(2) <= u && u <= l / T(2) && -w / T(2) <= v && v <= w / T(2)) return true;
    }
  }
  return false;
}

// IDM free-road term  COMFORT_ACC_MAX * (1 - (max(v,0)/|not_zero(v0)|)^DELTA)  (behavior.py:172-183),
// v0 = clip(target_speed, 0, speed_limit); idm_ratio is the power's base.
template <typename T>
__device__ __forceinline__ T idm_ratio(T v, T ts, T lim) {
  ts = clip(ts, T(0), lim);
  T vv = v;
  if (!(vv > T(0))) vv = (T(0) > vv) ? T(0) : vv;  // Python max(v, 0)
  return vv / fabs(not_zero(ts));
}
template <typename T, typename PP>
__device__ __forceinline__ T idm_free(const PP& P, T v, T ts, T lim, T delta) {
  return T(P.comfort_acc_max) * (T(1) - k_pow(idm_ratio(v, ts, lim), delta));
}
// The power split in two, so a vehicle's base can be shared: the act phase stores every vehicle's
// pow_base (float64: log of the ratio, as k_pow = exp(DELTA log ratio) computes it; float32: the
// ratio) and MOBIL's new-follower term raises it to the caller's DELTA with the same bits.
__device__ __forceinline__ double pow_base(double ratio) { return ttrl_math::log_d(ratio); }
__device__ __forceinline__ float pow_base(float ratio) { return ratio; }
__device__ __forceinline__ double pow_from_base(double b, double delta) { return ttrl_math::exp_d(delta * b); }
__device__ __forceinline__ float pow_from_base(float b, float delta) { return t_pow(b, delta); }

// IDM interaction term  COMFORT_ACC_MAX * (desired_gap(e, f) / not_zero(d))^2 (behavior.py:185-189,
// desired_gap :192-217, lane_distance_to objects.py:182-197 along e's current lane).
template <bool CV = true, typename T, typename PP>
__device__ __forceinline__ T idm_interact(const View<T>& V, const PP& P, int eb, int e, int f) {
  const LaneT<T> L = V.lanes[V.lane[eb + e]];
  T s1, r1, s0, r0;
  lane_local<CV>(L, V.x[eb + f], V.y[eb + f], s1, r1);
  lane_local<CV>(L, V.x[eb + e], V.y[eb + e], s0, r0);
  const T d = s1 - s0;
  const T ev = V.v[eb + e], ec = V.ch[eb + e], es = V.sh[eb + e];
  const T fv = V.v[eb + f], fc = V.ch[eb + f], fs = V.sh[eb + f];
  const T dvx = ev * ec - fv * fc, dvy = ev * es - fv * fs;
  const T dv = dvx * ec + dvy * es;
  const T gap = T(P.distance_wanted) + ev * T(P.time_wanted) + ev * dv / T(P.gap_denom);
  const T q = gap / not_zero(d);
  return T(P.comfort_acc_max) * (q * q);
}

// Full IDMVehicle.acceleration(ego=e, front=f) with the caller's DELTA (behavior.py:150-190).
template <bool CV = true, typename T, typename PP>
__device__ __forceinline__ T idm_acc(const View<T>& V, const PP& P, int eb, int e, int f, T delta) {
  if (e < 0) return T(0);
  const LaneT<T> L = V.lanes[V.lane[eb + e]];
  T a = idm_free(P, V.v[eb + e], V.ts[eb + e], L.lim, delta);
  if (f >= 0) a -= idm_interact<CV>(V, P, eb, e, f);
  return a;
}

// One pass answering up to 3 Road.neighbour_vehicles queries per thread (road.py:480-513)
// over the compacted per-lane candidate lists: front = min s_v >= s (ties: later slot),
// rear = max s_v < s (ties: earlier slot), visiting candidates in slot (= list) order.
// The entries of lane l's list (env le) from position `from` on, walked from the lane's on-lane
// slot mask in slot (= list) order with s recomputed by lane_local (the bits the projection
// stored), continuing a scan's front (s <= x <= sf: later wins ties) and rear (x < s, x > sr:
// earlier wins) updates, with slots in f / r.  The one-wavefront road network's rows hold
// GRAPH_LIST_CAP entries; longer lists are rare.
template <typename T, int NS>
__device__ __forceinline__ void overflow_scan(const View<T>& V, int le, int self, int l, int from, T s, T& sf, int& f,
                                           bool rear, T& sr, int& r) {
  constexpr unsigned long long SEG = NS == 64 ? ~0ull : ((1ull << NS) - 1);
  unsigned long long m = (V.onm[l] >> (le * NS)) & SEG;
  for (int c = 0; c < from && m; ++c) m &= m - 1;
  const LaneT<T> L = V.lanes[l];
  for (; m; m &= m - 1) {
    const int j = __builtin_ctzll(m);
    if (j == self) continue;
    T x, rr;
    lane_local<true>(L, V.x[le * NS + j], V.y[le * NS + j], x, rr);
    if (s <= x && x <= sf) { sf = x; f = j; }
    if (rear && x < s && x > sr) { sr = x; r = j; }
  }
}

// Bit q of RM asks for query q's rear (the caller may need only fronts).  The updates are
// selects, so the loop body is straight-line code.
template <typename T, int NQ, int NS, int EPW, unsigned RM = 7u, int LC = NS>
__device__ __forceinline__ void scan_neighbours(const View<T>& V, int le, int self, const int (&ql)[NQ],
                                                const T (&s)[NQ], int (&f)[NQ], int (&r)[NQ]) {
  constexpr int NSP = LC + 1;
  const int* cnt = V.cnt + le * (LMAX + 1);
  const int mx = cnt[LMAX] < LC ? cnt[LMAX] : LC;
  T sf[NQ], sr[NQ];
  int n[NQ], me[NQ], fp[NQ], rp[NQ];
  const T* row[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    sf[q] = K<T>::inf(); sr[q] = -K<T>::inf(); fp[q] = -1; rp[q] = -1;
    const int l = ql[q] < 0 ? 0 : ql[q];
    row[q] = V.key + ((size_t)l * EPW + le) * NSP;
    n[q] = ql[q] < 0 ? 0 : (cnt[l] < LC ? cnt[l] : LC);
    me[q] = V.mypos[(size_t)l * EPW * NS + le * NS + self];  // self is skipped by position
  }
  constexpr int U = NQ == 1 ? 8 : 4;
  for (int k0 = 0; k0 < mx; k0 += U) {
    T sv[NQ][U];
#pragma unroll
    for (int q = 0; q < NQ; ++q)
#pragma unroll
      for (int u = 0; u < U; ++u) sv[q][u] = row[q][k0 + u];
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const int kk = k0 + u;
        const T x = sv[q][u];
        const bool ok = kk < n[q] && kk != me[q];
        const bool uf = ok && s[q] <= x && x <= sf[q];
        sf[q] = uf ? x : sf[q];
        fp[q] = uf ? kk : fp[q];
        if (RM & (1u << q)) {
          const bool ur = ok && x < s[q] && x > sr[q];
          sr[q] = ur ? x : sr[q];
          rp[q] = ur ? kk : rp[q];
        }
      }
    }
  }
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const uint8_t* ix = V.idx + ((size_t)(ql[q] < 0 ? 0 : ql[q]) * EPW + le) * NSP;
    f[q] = fp[q] >= 0 ? (int)ix[fp[q]] : -1;
    r[q] = rp[q] >= 0 ? (int)ix[rp[q]] : -1;
  }
  if constexpr (LC < NS) {  // lists beyond the row capacity: the rest, in list order, from the lane mask
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      if (ql[q] < 0 || cnt[ql[q]] <= LC) continue;
      overflow_scan<T, NS>(V, le, self, ql[q], LC, s[q], sf[q], f[q], (RM & (1u << q)) != 0, sr[q], r[q]);
    }
  }
}

enum { MODE_META = 1, MODE_ACT = 2, MODE_STEP = 4 };
// Diagnostic ablation bits (ttrl_diag_simulate only; results are then NOT the reference's).
enum { A_NO_COLL = 1, A_NO_MOBIL = 2, A_NO_ABORT = 4, A_NO_SCAN = 8, A_NO_STEER = 16, A_NO_KIN = 32,
       A_NO_LANE = 64, A_NO_IDM = 128, A_NO_SAT = 256, A_NO_PREF = 512,
       A_SAT_SERIAL = 1024 /* one pair per lane (sat_pair) instead of one axis per lane; same results */ };

enum { FL_CRASHED = 1, FL_IMPACT = 2, FL_LC = 4, FL_YIELD = 8 };


// Diagnostic builds only.  -DTTRL_PHASE_TIMING: per-phase shader-clock cycles of every wave,
// summed into g_phase (tools/phases.py); the accumulators live in LDS (32-bit, one row per wave),
// so the stamps leave the kernel's register allocation as it is (a register array of 20 counters
// cost 40 VGPRs and spilled) -- but they add 320 B of LDS per workgroup.  -DTTRL_WAVE_TRACE: every
// wave's (start, end) shader clock with its HW_ID / XCC_ID, no LDS (tools/phases.py --waves).
// The production kernel carries neither.
#if defined(TTRL_PHASE_TIMING) || defined(TTRL_WAVE_TRACE)
__device__ unsigned long long g_phase[PH_SLOTS];  // 20 phases, project_items' and the regulation's steps
constexpr int WTRACE_MAX = 16384;
__device__ unsigned long long g_wtrace[WTRACE_MAX][3];
__device__ unsigned g_wphase[WTRACE_MAX][PH_SLOTS];  // PHASE_TIMING: each wave's phase cycles of the last launch
#define WT_INIT const unsigned long long ph_t0 = __builtin_readcyclecounter();
#define WT_FLUSH                                                       \
  {                                                                    \
    const unsigned ph_w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); \
    if ((threadIdx.x & 63) == 0 && ph_w < WTRACE_MAX) {                \
      g_wtrace[ph_w][0] = ph_t0;                                       \
      g_wtrace[ph_w][1] = __builtin_readcyclecounter();                \
      g_wtrace[ph_w][2] = ((unsigned long long)__builtin_amdgcn_s_getreg(63508) << 32) | __builtin_amdgcn_s_getreg(63492); \
    }                                                                  \
  }
#endif
#ifdef TTRL_PHASE_TIMING
#define PH_INIT                                                        \
  WT_INIT                                                              \
  if ((threadIdx.x & 63) < PH_SLOTS) ph_acc[threadIdx.x >> 6][threadIdx.x & 63] = 0; \
  unsigned long long ph_t = ph_t0;
#define PH(k)                                                          \
  do {                                                                 \
    const unsigned long long ph_n = __builtin_readcyclecounter();      \
    if ((threadIdx.x & 63) == 0) ph_acc[threadIdx.x >> 6][k] += (unsigned)(ph_n - ph_t); \
    ph_t = ph_n;                                                       \
  } while (0)
#define PH_FLUSH                                                       \
  if ((threadIdx.x & 63) < PH_SLOTS) {                                 \
    atomicAdd(&g_phase[threadIdx.x & 63], (unsigned long long)ph_acc[threadIdx.x >> 6][threadIdx.x & 63]); \
    const unsigned ph_w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); \
    if (ph_w < WTRACE_MAX) g_wphase[ph_w][threadIdx.x & 63] = ph_acc[threadIdx.x >> 6][threadIdx.x & 63]; \
  }                                                                    \
  WT_FLUSH
#elif defined(TTRL_WAVE_TRACE)
#define PH_INIT WT_INIT
#define PH(k)
#define PH_FLUSH WT_FLUSH
#else
#define PH_INIT
#define PH(k)
#define PH_FLUSH
#endif

template <typename T, int NS, int EPW, typename EgoFn, typename PP>
__device__ __forceinline__ void kin_observe(const ttrl_state_t& st, const LaneT<T>* lanes, const PP& P,
                                            const ttrl_kin_cfg_t& cfg, bool env_ok, int env, T x, T y, T h, T v,
                                            T hc, T hs, int lane, bool present, bool mdp, EgoFn ego_of, T* s_key,
                                            int* s_cnt, int* s_ego, int (*s_perm)[64], int (*s_p)[64],
                                            float* __restrict__ out, int32_t* __restrict__ ids,
                                            float* __restrict__ out2 = nullptr, int32_t* __restrict__ ids2 = nullptr);
template <typename T>
__device__ __forceinline__ void step_tail(const ttrl_lane_table_t& R, const LaneT<T>* L, const ttrl_reward_cfg_t& cfg,
                                          int env, bool has_ego, T x, T y, T v, int l, bool crashed, T v0,
                                          bool crashed0, double* __restrict__ time, double time_inc,
                                          float* __restrict__ reward, uint8_t* __restrict__ term,
                                          uint8_t* __restrict__ trunc, float* __restrict__ comp,
                                          T* __restrict__ ego_speed, uint8_t* __restrict__ ego_crashed);

// What ttrl_env_step adds after the last frame (null pointers: nothing): the Kinematics observation
// of the final state and the step tail of ttrl_rewards_step (time, reward, terminated, truncated,
// reward components, the info's ego speed / crashed), both from the on-chip view.
// Scratch of grid_observe (LDS): per-cell winners, the on_road bitmap, the clipped feature values
// per vehicle, and the observer passed through LDS.
template <typename T> struct GridScr {
  int* win;         // [C] winner vehicle index
  unsigned* road;   // [ceil(C/32)] on_road bitmap
  float* val;       // [F][N] clipped feature values
  int* ego;         // [1] the observer's slot
  T* e;             // [6] its x, y, heading, speed, cos, sin
  int* elane;       // [1] its lane
};
__host__ __device__ inline size_t grid_scratch_bytes(const ttrl_grid_cfg_t& cfg, int N, size_t real) {
  const size_t C = (size_t)cfg.shape_x * cfg.shape_y;
  return ((4 * C + 4 * ((C + 31) / 32) + 15) & ~(size_t)15) + ((4 * (size_t)cfg.n_features * N + 15) & ~(size_t)15) +
         6 * real + 16;
}
template <typename T>
__device__ __forceinline__ GridScr<T> grid_scratch(char* base, const ttrl_grid_cfg_t& cfg, int N) {
  const int C = cfg.shape_x * cfg.shape_y;
  GridScr<T> g;
  g.win = (int*)base;
  g.road = (unsigned*)(g.win + C);
  g.val = (float*)(base + ((4 * (size_t)C + 4 * (size_t)((C + 31) / 32) + 15) & ~(size_t)15));
  g.e = (T*)((char*)g.val + ((4 * (size_t)cfg.n_features * N + 15) & ~(size_t)15));
  g.ego = (int*)(g.e + 6);
  g.elane = g.ego + 1;
  return g;
}

template <typename T, typename KindOf, typename VehOf>
__device__ __forceinline__ void grid_observe(const ttrl_lane_table_t& R, const ttrl_grid_cfg_t& cfg, int N, int tid,
                                             int nt, int kd, T x, T y, T h, T v, T hc, T hs, int ln, KindOf kind_of,
                                             VehOf veh_of, const GridScr<T>& g, float* __restrict__ ob,
                                             bool nt_stores = true);

// The fused launch's grid write-out: nontemporal stores (1: 0.580 against 0.583 ms per config-3
// step with plain ones, profiles/r06/r06i_*)
#ifndef TTRL_GRID_NT_STORES
#define TTRL_GRID_NT_STORES 1
#endif
// ttrl_env_step_grid's epilogue: the OccupancyGrid of the final state, with grid_observe's scratch
// at byte `scr` of the view's LDS block (over the blocks dead after the last frame)
struct GridEpi {
  ttrl_grid_cfg_t cfg;
  float* out;
  uint32_t scr;
};
// simulate_body's epilogues: the state store + ttrl_env_step's tail; + the OccupancyGrid; the
// intersection's (ix_epilogue)
constexpr int EPI_STEP = 0, EPI_GRID = 1, EPI_IX = 2;

struct StepOut {
  ttrl_kin_cfg_t kcfg;
  float* obs;
  int32_t* ids;
  ttrl_reward_cfg_t rcfg;
  double* time;
  double time_inc;
  float* reward;
  uint8_t *term, *trunc;
  float* comp;
  void* ego_speed;
  uint8_t* ego_crashed;
  // workgroup slot -> env (a permutation of the envs, EPW consecutive entries per workgroup; a
  // negative entry: an idle slot; null: slot order).  A dispatch order only: every env's result is
  // independent of it.  It must not name an env twice (two workgroups would write one env).
  const int32_t* order;
  // n_lut > 0: actions[] are action indices, mapped to meta-action codes by lut (an index outside
  // the table: no meta-action)
  int8_t lut[8];
  int32_t n_lut;
};

// The env of workgroup slot q: order[q] under a dispatch order, else q; -1 (no env) for slots at or
// past qend (the last workgroup of an odd batch).
__device__ __forceinline__ int env_at(const int32_t* order, int q, int qend) {
  return q < qend ? (order ? order[q] : q) : -1;
}

// A per-vehicle value only its own thread reads: a register, or (L) its slot in an LDS view array.
template <bool L, typename T> struct Own {
  T r;
  T* p;
  __device__ __forceinline__ operator T() const {
    if constexpr (L) return *p;
    else return r;
  }
  __device__ __forceinline__ Own& operator=(T v) {
    if constexpr (L) *p = v;
    else r = v;
    return *this;
  }
};

// ttrl_ix_env_step: IntersectionEnv.step's tail (_clear_vehicles, _spawn_vehicle;
// intersection_env.py:135-139, 320-362) fused into the step launch for the envs that go on
// (neither terminated nor truncated), on their LDS rows after the step tail (ix_epilogue).  The
// finished envs are left to ttrl_ix_step_tail (cleared = 1), which swaps in their spare scenes.
struct IxEpi {
  ttrl_ix_cfg_t C;
  double lane_change_delay;  // ttrl_params_t's, float64 as in the scene kernels (a spawn's IDM timer)
  float* obs2;               // [E, V, F]: the next observation (an env that goes on keeps this step's)
  int32_t* ids2;             // [E, V - 1] (or null)
  unsigned long long* live;  // optional: += the vehicles present after the tail
  int32_t* live_env;         // optional [E]: each env's vehicles present after the tail (ix_order_kernel)
  // the auto-reset from scenes reset ahead of time (ttrl_ix_step_tail's, see there): a finished env
  // takes spare row par[e] * E + e
  ttrl_state_t spare;        // K * E rows
  int K;
  uint8_t* par;              // [E]
  uint32_t* ent;             // [E][nw], the episode counter last
  uint32_t* spare_ent;       // [K * E][nw]
  int nw;
  uint8_t* done;             // [E] out
  uint8_t* spare_mask;       // [K * E] out
};

template <typename T, int NS, int EPW>
__device__ __forceinline__ void ix_epilogue(const View<T>& V, const ttrl_state_t& st, const ttrl_lane_table_t& R,
                                            const ParamsT<T>& P, const StepOut& so, const IxEpi& ie, int le, int i,
                                            int env, bool env_on, bool slot, size_t k, int me, int eb, int reg,
                                            T& timer, T& steer, T& acc, T& ix, T& iy, int& sidx);

// Fused frame loop.  EPW envs per workgroup, NS slots per env, blockDim = EPW*NS.  The whole
// vehicle state of the workgroup's envs is resident in LDS for the launch (HBM is read once
// and written once); each phase loads the few fields it needs into registers, so no state is
// live across phases and the kernel runs at high occupancy without spilling.  The workgroup
// takes the envs of slots [q0, q0 + EPW) (below qend) of the dispatch order (simulate_kernel:
// q0 = blockIdx.x * EPW, qend = n_envs).  EPI: the epilogue (EPI_GRID: + the OccupancyGrid, ge;
// EPI_IX: ix_epilogue, ie).
template <typename T, int NS, int EPW, int NET, int EPI = EPI_STEP>
__device__ __forceinline__ void simulate_body(int q0, int qend, const ttrl_state_t& st, const ttrl_lane_table_t& R,
                                              const ParamsT<T>& P, const int32_t* __restrict__ actions,
                                              const uint8_t* __restrict__ env_mask, int frames, double dt_d, int mode,
                                              int ablate_arg, const StepOut& so, const IxEpi* ie = nullptr,
                                              const GridEpi* ge = nullptr);

template <typename T, int NS, int EPW, int NET, int WB = 0>
// Waves per SIMD the register budget is sized for: 4 on the straight highway (its compile-time
// LDS view, <= 10 KB per 64-slot env in float64, fits 4 workgroups per SIMD, so a 4096-env batch
// runs in one round instead of two: 0.455 -> 0.356 ms per float64 launch with machine LICM off,
// see build flags), 2 on curved roads in float64 and on a road network (whose LDS view allows
// ~1.25-2.5 waves per SIMD anyway).  WB > 0 overrides: the two-env-per-wave straight instance
// (NS = 32) has a 2-wave twin for batches whose waves all fit at 2 per SIMD (4096 32-slot envs
// are 2048 waves), where the 4-wave budget would spill for nothing (launch_sim).
__global__ void __launch_bounds__(NS* EPW, TTRL_SIM_WAVES > 0 ? TTRL_SIM_WAVES
                                               : WB > 0 ? WB
                                                        : (NET == NET_STRAIGHT ? 4
                                                                               : (sizeof(T) == 8 || NET == NET_GRAPH ? 2 : 4)))
simulate_kernel(ttrl_state_t st, ttrl_lane_table_t R, ParamsT<T> P, const int32_t* __restrict__ actions,
                const uint8_t* __restrict__ env_mask, int frames, double dt_d, int mode, int ablate_arg, StepOut so) {
  simulate_body<T, NS, EPW, NET>((int)blockIdx.x * EPW, st.n_envs, st, R, P, actions, env_mask, frames, dt_d, mode,
                                 ablate_arg, so);
}

// ttrl_ix_env_step: the road-network instance with IntersectionEnv.step's tail fused (IxEpi)
template <typename T, int NS, int EPW>
__global__ void __launch_bounds__(NS* EPW, TTRL_SIM_WAVES > 0 ? TTRL_SIM_WAVES : 2)
simulate_ix_kernel(ttrl_state_t st, ttrl_lane_table_t R, ParamsT<T> P, const int32_t* __restrict__ actions,
                   int frames, double dt_d, StepOut so, IxEpi ie) {
  simulate_body<T, NS, EPW, NET_GRAPH, EPI_IX>((int)blockIdx.x * EPW, st.n_envs, st, R, P, actions, nullptr, frames,
                                               dt_d, MODE_META | MODE_ACT | MODE_STEP, 0, so, &ie);
}

// ttrl_env_step_grid: the straight one-env-per-workgroup instance (sorted view) with the
// OccupancyGrid of the final state written by the launch (GridEpi)
template <typename T, int NS>
__global__ void __launch_bounds__(NS, TTRL_SIM_WAVES > 0 ? TTRL_SIM_WAVES : 4)
simulate_grid_kernel(ttrl_state_t st, ttrl_lane_table_t R, ParamsT<T> P, const int32_t* __restrict__ actions,
                     int frames, double dt_d, StepOut so, GridEpi ge) {
  simulate_body<T, NS, 1, NET_STRAIGHT, EPI_GRID>((int)blockIdx.x, st.n_envs, st, R, P, actions, nullptr, frames, dt_d,
                                                  MODE_META | MODE_ACT | MODE_STEP, 0, so, nullptr, &ge);
}

template <typename T, int NS, int EPW, int NET, int EPI>
__device__ __forceinline__ void simulate_body(int q0, int qend, const ttrl_state_t& st, const ttrl_lane_table_t& R,
                                              const ParamsT<T>& P, const int32_t* __restrict__ actions,
                                              const uint8_t* __restrict__ env_mask, int frames, double dt_d, int mode,
                                              int ablate_arg, const StepOut& so, const IxEpi* ie, const GridEpi* ge) {
  // The diagnostic phase ablations (ttrl_diag_simulate) exist only in -DTTRL_DIAG_ABLATE builds: as a
  // run-time argument their ~20 tests held SGPR masks for the whole launch (spilled to VGPR lanes),
  // and the product passes 0 anyway.
#ifdef TTRL_DIAG_ABLATE
  const int ablate = ablate_arg;
#else
  constexpr int ablate = 0;
  (void)ablate_arg;
#endif
  constexpr bool CV = NET != NET_STRAIGHT;  // curved lane classes possible
  constexpr bool GR = NET == NET_GRAPH;     // roads, routes, RegulatedRoad
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NT = NS * EPW;
  constexpr int WAVES = NT / 64 > 0 ? NT / 64 : 1;
  const int tid = threadIdx.x;
  const int le = tid / NS, i = tid % NS;
  const int N = st.n_veh, nl = R.n_lanes;
  // road networks take their envs in so.order (heaviest workgroups first, see ix_order_kernel)
  const int32_t* ord = GR ? so.order : nullptr;
  const int env = env_at(ord, q0 + le, qend);
  const bool env_on = (unsigned)env < (unsigned)st.n_envs && (!env_mask || env_mask[env]);  // masked-out envs: untouched
  if (env_mask) {  // a workgroup with no active env leaves at once (uniform: before any barrier)
    bool any = false;
    for (int q = 0; q < EPW; ++q) {
      const int e = env_at(ord, q0 + q, qend);
      any |= (unsigned)e < (unsigned)st.n_envs && env_mask[e];
    }
    if (!any) return;
  }
  const bool slot = env_on && i < N;
  const size_t k = (size_t)env * N + i;
  const int me = le * NS + i;  // this vehicle's LDS slot
  const int eb = le * NS;      // env base in the LDS view
  // The straight-road instance carves a compile-time layout (LANE_CAP lanes): every view array
  // is then the LDS base plus an immediate offset, so no base addresses occupy registers.
  constexpr bool SO = sorted_view(NS, EPW, NET);
  constexpr int LC = list_cap(NS, EPW, GR);  // list row capacity (GRAPH_LIST_CAP on one-wave networks)
  View<T> V = carve<T>(smem, EPW, NS, NET == NET_STRAIGHT ? STRAIGHT_LANE_CAP : nl, GR, SO);
  PH_INIT
  stage_lanes(V, R, tid);
  if constexpr (GR) {
    if (tid < TTRL_MAX_ROADS) {
      V.rt->from[tid] = R.road_from[tid]; V.rt->to[tid] = R.road_to[tid];
      V.rt->first[tid] = R.road_first[tid]; V.rt->n[tid] = R.road_n[tid];
    }
    if (tid == 0) V.rt->n_roads = R.n_roads;
    // project_items' lane order: straight lanes first, then the curved ones (list order within)
    const bool cur = tid < nl && V.lanes[tid].type != TTRL_LANE_STRAIGHT;
    const unsigned long long below = (1ull << (tid & 63)) - 1;
    const unsigned long long cm = __ballot(cur), sm = __ballot(tid < nl && !cur);
    if (tid < nl) V.lperm[cur ? __popcll(sm) + __popcll(cm & below) : __popcll(sm & below)] = (int8_t)tid;
  }
  const T dt = T(dt_d);

  bool present;
  // Vehicle state only this thread reads (IDM timer, the action, the pending impact) stays in
  // registers for the launch; what other vehicles read is staged in the LDS view.
  T my_timer;
  // the action and the pending impact: LDS on the sorted (4 waves per SIMD) instance, see view_layout
  Own<SO, T> my_steer{T(0), SO ? V.steer + me : nullptr}, my_acc{T(0), SO ? V.acc + me : nullptr},
      my_ix{T(0), SO ? V.ix + me : nullptr}, my_iy{T(0), SO ? V.iy + me : nullptr};
  int my_sidx;
  int my_sorted = 0;  // SO: the slot at this lane's sorted position
  {  // HBM -> LDS, once per launch (coalesced SoA rows)
    Veh<T> a;
    if (slot) load_veh(a, st, k);
    else { a = Veh<T>{}; a.kind = TTRL_ABSENT; a.lane = -1; a.tgt = -1; }
    present = slot && a.kind != TTRL_ABSENT;
    V.x[me] = present ? a.x : T(FAR); V.y[me] = a.y;
    if constexpr (sizeof(T) == 8) V.xf[me] = present ? (float)a.x : FAR; V.v[me] = a.v; V.ts[me] = a.ts;
    const SinCos<T> sc = k_sincos(a.h);
    V.ch[me] = sc.c; V.sh[me] = sc.s;
    V.h[me] = a.h; V.delta[me] = a.delta;
    my_timer = a.timer; my_steer = a.steer; my_acc = a.acc; my_ix = a.ix; my_iy = a.iy;
    V.kind[me] = (uint8_t)(present ? a.kind : TTRL_ABSENT);
    V.flags[me] = (uint8_t)((a.crashed ? FL_CRASHED : 0) | (a.hasimp ? FL_IMPACT : 0) | (a.lc ? FL_LC : 0));
    my_sidx = a.sidx;
    V.lane[me] = (int8_t)(present ? a.lane : -1);
    V.tgt[me] = (int8_t)(present ? a.tgt : -1);
    if constexpr (GR) {
      for (int q = 0; q < TTRL_ROUTE_MAX; ++q) {
        V.rroad[me * TTRL_ROUTE_MAX + q] = slot ? st.route_road[k * TTRL_ROUTE_MAX + q] : (int8_t)-1;
        V.rlane[me * TTRL_ROUTE_MAX + q] = slot ? st.route_lane[k * TTRL_ROUTE_MAX + q] : (int8_t)-1;
      }
      V.rn[me] = slot ? st.route_n[k] : (int8_t)-1;
      if (slot && st.yielding[k]) V.flags[me] |= FL_YIELD;
    }
  }
  int reg = 0;  // RegulatedRoad.steps of this thread's env
  if constexpr (GR) reg = env_on ? st.reg_steps[env] : 0;
  const int reg_period = GR && R.regulation_frequency > 0 ? (int)(1.0 / dt_d / R.regulation_frequency) : 0;
  PH(15);
  if (i == 0) V.nitem[le] = 0;
  __syncthreads();  // lane table + view staged
  // project_items' pruning: each thread < nl keeps its lane's box for the launch; the on-lane reach
  // is the widest lane's w / 2 + 1 + LENGTH (AbstractLane.on_lane, margin 1)
  float4 my_box = make_float4(0.f, 0.f, 0.f, 0.f);
  float onb_all = 0.0f;
  if constexpr (GR && NS * EPW == 64) {
    if (tid < nl) my_box = lane_box(V.lanes[tid]);
    for (int l = 0; l < nl; ++l) onb_all = fmaxf(onb_all, (float)(R.width[l] / 2 + 1 + P.lane_vehicle_length));
  }
  {
    int ob = 0;
    const T x0 = V.x[me];
    project_all<T, NS, EPW, CV, !SO, LC>(V, P, nl, tid, le, i, present, x0, V.y[me], T(0), false, &ob);
    if constexpr (SO && NS == 128) sort_order128<T>(V, nl, tid, true, my_sorted);
    else if constexpr (SO) sort_order<T, NS, EPW>(V, nl, tid, le, i, true, my_sorted, x0, ob);
  }
  const int kind = V.kind[me];

  // ---------------- ego meta-action (DiscreteMetaAction.act, action.py:259-260) ----
  // PEEL (the 128 / 256-slot straight instances, road networks): the first frame's meta-action runs
  // before the frame loop (nothing of frame 0 runs before it), so the env index and the action's
  // address die there instead of living through the loop (at NS = 128 they were spilled to scratch),
  // and the ego's speed index is written to HBM where it changes (store_veh<false> at the end), not
  // held in a register to the end.  The 32 / 64-slot straight instances keep it inside the loop:
  // peeled, their launches measured ~1 % slower (profiles/r06/r06n).
  constexpr bool PEEL = NS > 64 || GR;
  auto meta_action = [&](int envl) {
    int act = actions[envl];
    if (so.n_lut > 0) {  // the env's action index -> its meta-action code (a select chain)
      int c = -1;
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (q < so.n_lut && act == q) c = so.lut[q];
      act = c;
    }
    const T x = V.x[me], y = V.y[me], h = V.h[me], v = V.v[me];
    T ts = V.ts[me];
    int tgt = V.tgt[me];
    if constexpr (GR)  // ControlledVehicle.act starts with follow_road (controller.py:98)
      tgt = follow_road(V.lanes, *V.rt, T(P.lane_vehicle_length), tgt, x, y, V.rroad + me * TTRL_ROUTE_MAX,
                        V.rlane + me * TTRL_ROUTE_MAX, V.rn + me, lane_s<T, NS, EPW, LC>(V, tgt, le, i, x, y));
    if (act == TTRL_FASTER || act == TTRL_SLOWER) {  // MDPVehicle.act controller.py:304-315
      int si = speed_to_index(P, v) + (act == TTRL_FASTER ? 1 : -1);
      si = si < 0 ? 0 : (si > P.n_target_speeds - 1 ? P.n_target_speeds - 1 : si);
      my_sidx = si;
      // the launch's own state write-back leaves the speed index alone (store_veh<false>): a
      // register held to the end for one ego per env was spilled to scratch (NS = 128)
      if constexpr (PEEL && EPI != EPI_IX) st.speed_index[k] = si;
      ts = T(P.target_speeds[si]);
    } else if (act == TTRL_LANE_LEFT || act == TTRL_LANE_RIGHT) {  // controller.py:103-124
      int id, lo = 0, hi = nl - 1;
      if constexpr (GR) {  // clip within the target's road
        const LaneT<T>& TL = V.lanes[tgt];
        lo = TL.rfirst; hi = TL.rfirst + TL.rn - 1;
      }
      id = tgt + (act == TTRL_LANE_RIGHT ? 1 : -1);
      id = id < lo ? lo : (id > hi ? hi : id);
      if (reachable<CV>(V.lanes[id], T(P.lane_vehicle_length), x, y)) tgt = id;
    }
    // ControlledVehicle.act low-level control (controller.py:126-133); Road.act recomputes
    // the same values this frame, the standalone ttrl_meta_action returns them.
    my_steer = steering_control<CV>(V.lanes[tgt], P, x, y, h, v);
    my_acc = T(P.kp_a) * (ts - v);
    V.ts[me] = ts;
    V.tgt[me] = (int8_t)tgt;
  };
  if constexpr (PEEL) {
    if ((mode & MODE_META) && frames > 0 && actions && present && kind == TTRL_MDP) meta_action(env);
  }

  // Fair issue among a SIMD's waves.  The SIMD's arbiter issues the oldest ready wave first, so the
  // first-dispatched of its waves ran ahead and the last one finished alone: on the headline launch
  // the four waves of a SIMD took 295 k / 348 k / 423 k / 511 k cycles by dispatch rank, the last
  // ~90 k of them one wave with no latency hiding (tools/placement.py, profiles/r06/
  // r06l_wave_placement.txt).  A wave's priority now falls with its progress, 3 in the first
  // quarter of the frames ... 0 in the last: a wave that is ahead yields to the ones behind it, so
  // the SIMD's waves stay together and finish close together (385 k / 408 k / 430 k / 451 k;
  // profiles/r06/r06r).  The straight instances with <= 64 slots only: the 128-slot one (two rounds
  // of two-wave workgroups) measured 5 % slower with it, and the road-network step launch 0.494 ms
  // per step with it and without (profiles/r06/r06s).  Masked launches (the intersection's
  // spare-reset warm-ups) keep the default priority.
  constexpr bool FAIR = NS <= 64 && !GR;
  const bool fair = FAIR && !env_mask && frames >= 4;
  if (fair) __builtin_amdgcn_s_setprio(3);
  PH(11);
  for (int frame = 0; frame < frames; ++frame) {
    if (fair && frame > 0) {
      const int q = frame * 4 / frames, qp = (frame - 1) * 4 / frames;
      if (q != qp) {
        if (q == 1) __builtin_amdgcn_s_setprio(2);
        else if (q == 2) __builtin_amdgcn_s_setprio(1);
        else __builtin_amdgcn_s_setprio(0);
      }
    }
    if constexpr (!PEEL) {
      if ((mode & MODE_META) && frame == 0 && actions && present && kind == TTRL_MDP) meta_action(env);
    }
    __syncthreads();
    PH(0);

    // ---------------- Road.act (road.py:461-464) ----------------
    int tgt_new = V.tgt[me];
    const int tgt0 = tgt_new;  // the target before this vehicle's act (what earlier vehicles saw)
    if (mode & MODE_ACT) {
      const bool polite = P.politeness != 0.0;
      {  // (1) per vehicle: lane-change timer, own-lane (+ target-lane) neighbours, IDM free
         //     term, MOBIL work items; results go to LDS so nothing stays live across (2)
        if constexpr (GR) {  // follow_road opens IDMVehicle.act (not crashed) and ControlledVehicle.act
          if (present && (kind == TTRL_MDP || !(V.flags[me] & FL_CRASHED))) {
            tgt_new = follow_road(V.lanes, *V.rt, T(P.lane_vehicle_length), tgt_new, V.x[me], V.y[me],
                                  V.rroad + me * TTRL_ROUTE_MAX, V.rlane + me * TTRL_ROUTE_MAX, V.rn + me,
                                  lane_s<T, NS, EPW, LC>(V, tgt_new, le, i, V.x[me], V.y[me]));
            V.tgt[me] = (int8_t)tgt_new;
          }
        }
        PH(19);
        const int lane = V.lane[me], tgt = V.tgt[me];
        const int fl = V.flags[me];
        const bool idm = present && kind == TTRL_IDM && !(fl & FL_CRASHED);
        const bool lc = (fl & FL_LC) != 0;
        const bool changing = idm && lane != tgt;
        const T x = V.x[me], y = V.y[me], v = V.v[me];
        bool fire = false;
        if (idm && lc && !changing && T(P.lane_change_delay) < my_timer && !(ablate & A_NO_MOBIL)) {
          fire = true;  // utils.do_every
          my_timer = T(0);
        }
        // side lanes (RoadNetwork.side_lanes road.py:200-211), gated as behavior.py:252-260
        bool left = false, right = false;
        if (fire) {
          const bool moving = !(fabs(v) < T(1));
          bool has_l = lane > 0, has_r = lane < nl - 1;
          if constexpr (GR) {
            const LaneT<T>& OL = V.lanes[lane];
            has_l = OL.lid > 0;
            has_r = OL.lid < OL.rn - 1;
          }
          left = has_l && moving && reachable<CV>(V.lanes[lane - 1], T(P.lane_vehicle_length), x, y);
          right = has_r && moving && reachable<CV>(V.lanes[lane + 1], T(P.lane_vehicle_length), x, y);
        }
        // Queries of every vehicle: the own lane's front (its rear only feeds MOBIL's politeness
        // term) and, while changing lane, the target lane's front (IDMVehicle.act behavior.py:118-131).
        const int ql[2] = {idm ? lane : -1, changing ? tgt : -1};
        T s2[2];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          if constexpr (GR) {
            s2[q] = lane_s<T, NS, EPW, LC>(V, ql[q] < 0 ? 0 : ql[q], le, i, x, y);
          } else {
            T rr;
            lane_local<CV>(V.lanes[ql[q] < 0 ? 0 : ql[q]], x, y, s2[q], rr);
          }
        }
        int f2[2] = {-1, -1}, r2[2] = {-1, -1};
        PH(1);
        if constexpr (SO) {
          if (!(ablate & A_NO_SCAN)) {
            const bool tie = V.stie[le] != 0;
            const int p = V.spos[me];
#pragma unroll
            for (int q = 0; q < 2; ++q)
              if (ql[q] >= 0) {
                if (!tie) sorted_nbrs<T, NS>(V, le, ql[q], p, f2[q], r2[q]);
                else slot_nbrs<T, NS>(V, le, i, ql[q], s2[q], f2[q], r2[q]);
              }
          }
        } else if (!(ablate & A_NO_SCAN)) {
          if (__any(ql[1] >= 0)) {
            if (polite) scan_neighbours<T, 2, NS, EPW, 1u, LC>(V, le, i, ql, s2, f2, r2);
            else scan_neighbours<T, 2, NS, EPW, 0u, LC>(V, le, i, ql, s2, f2, r2);
          } else {
            const int ql1[1] = {ql[0]};
            const T s1[1] = {s2[0]};
            int f1[1], r1[1];
            if (polite) scan_neighbours<T, 1, NS, EPW, 1u, LC>(V, le, i, ql1, s1, f1, r1);
            else scan_neighbours<T, 1, NS, EPW, 0u, LC>(V, le, i, ql1, s1, f1, r1);
            f2[0] = f1[0]; r2[0] = r1[0];
          }
        }
        PH(2);
        T a_free = T(0);
        // IDM free-road term (behavior.py:172-183); the power's base of every present vehicle goes
        // to LDS for the MOBIL items (a new follower may be any vehicle, the caller's DELTA)
        const T pb = pow_base(idm_ratio(v, V.ts[me], V.lanes[lane < 0 ? 0 : lane].lim));
        V.powb[me] = pb;
        if (idm && !(ablate & A_NO_IDM)) a_free = T(P.comfort_acc_max) * (T(1) - pow_from_base(pb, V.delta[me]));
        PH(12);
        V.afree[me] = a_free;
        V.f0[me] = (short)f2[0];
        V.r0[me] = (short)r2[0];
        V.ft[me] = (short)f2[1];
        V.mob[me] = -3;            // -3: no item for this side
        V.mob[EPW * NS + me] = -3;
        // MOBIL (IDMVehicle.mobil behavior.py:265-324, route None) as work items, one per
        // (firing vehicle, candidate side lane): a frame has a handful of firing vehicles, so
        // the side-lane queries and IDM terms of all of them cost one pass.
        if constexpr (NS <= 64) {  // one wavefront: queue slots from ballots, no LDS atomics
          const int sh = (tid & 63) / NS * NS;
          const unsigned long long seg = NS == 64 ? ~0ull : ((1ull << NS) - 1) << sh;
          const unsigned long long below = (1ull << (tid & 63)) - 1;
          const unsigned long long bl = __ballot(left) & seg, br = __ballot(right) & seg;
          const int pos = __popcll(bl & below) + __popcll(br & below);
          if (left) V.item[le * 2 * NS + pos] = (short)i;
          if (right) V.item[le * 2 * NS + pos + (left ? 1 : 0)] = (short)(i | 0x4000);
          if (i == 0) V.nitem[le] = __popcll(bl) + __popcll(br);
        } else {
          if (left) V.item[le * 2 * NS + atomicAdd(&V.nitem[le], 1)] = (short)i;
          if (right) V.item[le * 2 * NS + atomicAdd(&V.nitem[le], 1)] = (short)(i | 0x4000);
        }
      }
      __syncthreads();
      PH(13);
      {  // (2) MOBIL items
        const int nitem = V.nitem[le];
        // G lanes per item: each scans every G-th candidate of the side lane's list, the group
        // combines (front: min s, ties to the later position; rear: max s, ties to the earlier),
        // then lanes 0-2 of the group evaluate the three IDM interaction terms side by side.
        constexpr int G = 8, IPP = NS / G;
        const int g = i % G;
        for (int t0 = 0; t0 < nitem; t0 += IPP) {
          const int t = t0 + i / G;
          if (t < nitem) {  // whole groups are active or idle together
            const int it = V.item[le * 2 * NS + t];
            const int side = it >> 14, vi = it & 0x3fff, ve = eb + vi;
            const int ln = V.lane[ve] + (side ? 1 : -1);
            T sq, rr;
            lane_local<CV>(V.lanes[ln], V.x[ve], V.y[ve], sq, rr);
            T sf = K<T>::inf(), sr = -K<T>::inf();
            int fp = -1, rp = -1;
            int np_ = -1, nf = -1;  // the side lane's front / rear of the item's vehicle
            const size_t rowb = SO ? 0 : ((size_t)ln * EPW + le) * (LC + 1);
            if constexpr (SO) {
              if (!(ablate & A_NO_SCAN)) {
                if (V.stie[le] == 0) sorted_nbrs<T, NS>(V, le, ln, V.spos[ve], np_, nf);
                else slot_nbrs<T, NS>(V, le, vi, ln, sq, np_, nf);
              }
            } else if (!(ablate & A_NO_SCAN)) {
              const T* row = V.key + rowb;
              const int n = V.cnt[le * (LMAX + 1) + ln] < LC ? V.cnt[le * (LMAX + 1) + ln] : LC;
              const int mep = V.mypos[(size_t)ln * EPW * NS + le * NS + vi];  // the item's vehicle is skipped
              for (int kk = g; kk < n; kk += G) {
                const T xk = row[kk];
                const bool uf = kk != mep && sq <= xk && xk <= sf;
                sf = uf ? xk : sf;
                fp = uf ? kk : fp;
                const bool ur = kk != mep && xk < sq && xk > sr;
                sr = ur ? xk : sr;
                rp = ur ? kk : rp;
              }
              // combine the group's 8 partial scans (front: min s, ties to the later position; rear:
              // max s, ties to the earlier), lane g with g ^ 1, g ^ 2, then 7 - g
              auto merge = [&](T osf, int ofp, T osr, int orp) {
                if (osf < sf || (osf == sf && ofp > fp)) { sf = osf; fp = ofp; }
                if (osr > sr || (osr == sr && orp >= 0 && (rp < 0 || orp < rp))) { sr = osr; rp = orp; }
              };
              merge(grp8_swap<1>(sf), grp8_swap<1>(fp), grp8_swap<1>(sr), grp8_swap<1>(rp));
              merge(grp8_swap<2>(sf), grp8_swap<2>(fp), grp8_swap<2>(sr), grp8_swap<2>(rp));
              merge(grp8_swap<4>(sf), grp8_swap<4>(fp), grp8_swap<4>(sr), grp8_swap<4>(rp));
            }
            if constexpr (!SO) {
              np_ = fp >= 0 ? (int)V.idx[rowb + fp] : -1;
              nf = rp >= 0 ? (int)V.idx[rowb + rp] : -1;
              if constexpr (LC < NS) {  // the list beyond the row capacity (every lane of the group alike)
                if (!(ablate & A_NO_SCAN) && V.cnt[le * (LMAX + 1) + ln] > LC)
                  overflow_scan<T, NS>(V, le, vi, ln, LC, sq, sf, np_, true, sr, nf);
              }
            }
            const int op = V.f0[ve], of = V.r0[ve];
            const T delta = V.delta[ve];
            // IDM_self(new follower, front = self), a(self | new front), a(self | old front): DELTA is the caller's
            const int e_ = g == 0 ? nf : (g <= 2 ? vi : -1);
            const int f_ = g == 0 ? vi : (g == 1 ? np_ : op);
            T term = T(0);
            if (e_ >= 0 && f_ >= 0) term = idm_interact<CV>(V, P, eb, e_, f_);
            T fr = T(0);
            if (g == 0 && nf >= 0) fr = T(P.comfort_acc_max) * (T(1) - pow_from_base(V.powb[eb + nf], delta));
            const T t_np = grp8_swap<1>(term), t_op = grp8_swap<2>(term);
            if (g == 0) {
              const T af = V.afree[ve];
              const T nfpa = nf >= 0 ? fr - term : T(0);
              bool ok = !(nfpa < -T(P.lane_change_max_braking));
              bool planned = false;  // a route with a planned lane (behavior.py:296-304)
              if constexpr (GR) planned = V.rn[ve] > 0 && V.rlane[ve * TTRL_ROUTE_MAX] >= 0;
              if (ok && planned) {
                T spa = af;
                if (np_ >= 0) spa -= t_np;
                const int tid_ = V.lanes[V.tgt[ve]].lid, cid = V.lanes[ln].lid, rid = V.rlane[ve * TTRL_ROUTE_MAX];
                const int s1 = (cid > tid_) - (cid < tid_), s2 = (rid > tid_) - (rid < tid_);
                if (s1 != s2 || spa < -T(P.lane_change_max_braking)) ok = false;
              } else if (ok) {
                T spa = af, sa = af;
                if (np_ >= 0) spa -= t_np;
                if (op >= 0) sa -= t_op;
                T jerk;
                if (polite) {
                  const T nfa = idm_acc<CV>(V, P, eb, nf, np_, delta);
                  const T ofa = idm_acc<CV>(V, P, eb, of, vi, delta);
                  const T ofpa = idm_acc<CV>(V, P, eb, of, op, delta);
                  jerk = spa - sa + T(P.politeness) * (nfpa - nfa + ofpa - ofa);
                } else {
                  jerk = spa - sa + T(P.politeness) * T(0);
                }
                if (jerk < T(P.lane_change_min_acc_gain)) ok = false;
              }
              V.mob[side * EPW * NS + ve] = (short)(ok ? np_ : -2);
            }
          }
        }
      }
      PH(14);
      __syncthreads();
      if (i == 0) V.nitem[le] = 0;
      // (3) per vehicle: MOBIL verdicts, lane-change abort, steering and IDM acceleration
      const int lane = V.lane[me], tgt = V.tgt[me];
      const int fl = V.flags[me];
      const bool idm = present && kind == TTRL_IDM && !(fl & FL_CRASHED);
      const bool changing = idm && lane != tgt;
      bool abort_cand = changing && (fl & FL_LC) != 0;
      if constexpr (GR) abort_cand = abort_cand && V.lanes[lane].road == V.lanes[tgt].road;  // behavior.py:231
      const T x = V.x[me], y = V.y[me], v = V.v[me];
      int side_front = -1;  // front on the lane MOBIL chose (left first, a later candidate overrides)
      const int mobl = V.mob[me], mobr = V.mob[EPW * NS + me];
      if (mobl >= -1) { tgt_new = lane - 1; side_front = mobl; }
      if (mobr >= -1) { tgt_new = lane + 1; side_front = mobr; }
      PH(3);
      // Lane-change abort in list order (behavior.py:229-244): vehicle i aborts if some
      // v != i with v.lane != T_i and v.target == T_i (v's target as of its own turn:
      // final for v < i, previous for v > i) is 0 < d(i->v) < d*(i, v).
      if (!(ablate & A_NO_ABORT)) {
        auto contributes = [&](int ii) -> bool {
          if (!present || ii == i) return false;
          const int Ti = V.tgt[eb + ii];
          const int tv = i < ii ? tgt_new : tgt0;
          if (!(lane != Ti && tv == Ti)) return false;
          const LaneT<T> L = V.lanes[V.lane[eb + ii]];
          T s1, r1, s0, r0;
          lane_local<CV>(L, x, y, s1, r1);
          lane_local<CV>(L, V.x[eb + ii], V.y[eb + ii], s0, r0);
          const T d = s1 - s0;
          const T ev = V.v[eb + ii], ec = V.ch[eb + ii], es = V.sh[eb + ii];
          const T dvx = ev * ec - v * V.ch[me], dvy = ev * es - v * V.sh[me];
          const T dv = dvx * ec + dvy * es;
          const T ds = T(P.distance_wanted) + ev * T(P.time_wanted) + ev * dv / T(P.gap_denom);
          return T(0) < d && d < ds;
        };
        if constexpr (NS <= 64) {
          const unsigned long long seg = NS == 64 ? ~0ull : ((1ull << NS) - 1);
          const int sh = (tid & 63) / NS * NS;
          unsigned long long mine = (__ballot(abort_cand) >> sh) & seg;
          while (__any(mine != 0)) {
            const int ii = mine ? __ffsll((long long)mine) - 1 : -1;
            const bool c = ii >= 0 && contributes(ii);
            const unsigned long long cb = (__ballot(c) >> sh) & seg;
            if (ii >= 0 && cb != 0 && i == ii) tgt_new = lane;
            if (mine) mine &= mine - 1;
          }
        } else {
          const int wave = tid >> 6;
          unsigned long long wb = __ballot(abort_cand);
          if ((tid & 63) == 0) V.bal[wave] = wb;
          __syncthreads();
          unsigned long long m[WAVES];
#pragma unroll
          for (int w = 0; w < WAVES; ++w) m[w] = V.bal[w];
          __syncthreads();
          int par = 0;
#pragma unroll
          for (int w = 0; w < WAVES; ++w) {
            while (m[w]) {
              const int ii = w * 64 + __ffsll((long long)m[w]) - 1;
              m[w] &= m[w] - 1;
              const unsigned long long cb = __ballot(contributes(ii));
              if ((tid & 63) == 0) V.bal[8 + par * 4 + wave] = cb;
              __syncthreads();
              bool any = false;
#pragma unroll
              for (int w2 = 0; w2 < WAVES; ++w2) any |= V.bal[8 + par * 4 + w2] != 0;
              if (any && i == ii) tgt_new = lane;
              par ^= 1;
            }
          }
        }
      }

      PH(4);
      // steering + IDM longitudinal (behavior.py:109-135); ego: ControlledVehicle.act (controller.py:126-133)
      const bool mdp = present && kind == TTRL_MDP;
      if (idm || mdp) {  // one steering pass for both kinds (the ego steers to its own target)
        const int sl = idm ? tgt_new : tgt;
        const LaneT<T>& SL = V.lanes[sl];
        T s, r;
        bool turn = false;
        if constexpr (!SO && CV) turn = SL.type == TTRL_LANE_CIRCULAR;
        if (turn) {
          if constexpr (!SO && CV) {
            // a turn: s from the lane's candidate list (the projection stored lane_local's s for this
            // position; lane_s recomputes it off the list), the lateral part as curved_local has it
            s = lane_s<T, NS, EPW, LC>(V, sl, le, i, x, y);
            const T dx = x - SL.cx, dy = y - SL.cy;
            r = SL.dirn * (SL.rad - sqrt(dx * dx + dy * dy));
          }
        } else {
          lane_local<CV>(SL, x, y, s, r);
        }
        // one steering evaluation for both branches (a divergent wave would run it twice)
        my_steer = (idm && (ablate & A_NO_STEER)) ? T(0) : steering_control_sr<CV>(SL, P, s, r, V.h[me], v);
      }
      if (idm) {
        const T a_free = V.afree[me];
        const int f0 = V.f0[me];
        T acc = a_free;
        if (f0 >= 0) acc -= idm_interact<CV>(V, P, eb, i, f0);
        if (lane != tgt_new) {
          const int ft = tgt_new == tgt ? (int)V.ft[me] : side_front;
          T a2 = a_free;
          if (ft >= 0) a2 -= idm_interact<CV>(V, P, eb, i, ft);
          if (a2 < acc) acc = a2;
        }
        my_acc = clip(acc, -T(P.acc_max), T(P.acc_max));
      } else if (mdp) {
        my_acc = T(P.kp_a) * (V.ts[me] - v);
      }
    }

    __syncthreads();  // act-phase readers of the old view are done
    PH(5);
    if (mode & MODE_ACT) V.tgt[me] = (int8_t)(present ? tgt_new : -1);

    // ---------------- Road.step(dt) (road.py:466-478) ----------------
    if (mode & MODE_STEP) {
      if constexpr (GR) {
        if (reg_period > 0) {  // RegulatedRoad.step regulation.py:28-32
          ++reg;
          const bool doreg = env_on && reg % reg_period == 0;
          if (__syncthreads_or(doreg)) {  // enforce_road_rules regulation.py:34-60, every env of the block in step
            if (doreg && present) {
              const int fl = V.flags[me];
              if (fl & FL_YIELD) {  // YIELD_DURATION = 0: last enforcement's yields end now
                V.ts[me] = V.lanes[V.lane[me]].lim;
                V.flags[me] = (uint8_t)(fl & ~FL_YIELD);
              }
              if constexpr (NS * EPW != 64)
                predict_poses(V.lanes, *V.rt, (int)V.lane[me], V.x[me], V.y[me], V.v[me], V.rroad + me * TTRL_ROUTE_MAX,
                              V.rlane + me * TTRL_ROUTE_MAX, (int)V.rn[me], V.px + me * PRED_T, V.py + me * PRED_T,
                              V.ps0 + me);
            }
            V.ynew[me] = 0;
            if constexpr (NS * EPW == 64) {
              // One wavefront: the predictions as (vehicle, time step) items over all its lanes (a scene
              // has ~8 live vehicles in 32 slots: one vehicle per lane walked its 11 poses serially)
              const bool pv = doreg && present;
              if (pv) {
                T s0, r0;
                lane_local(V.lanes[V.lane[me]], V.x[me], V.y[me], s0, r0);
                V.ps0[me] = s0;
              }
              const unsigned long long pm = __ballot(pv);
              if (pv) V.live[__popcll(pm & ((1ull << tid) - 1))] = (uint8_t)tid;
              __syncthreads();
              const int nitems = __popcll(pm) * PRED_T;
              for (int q = tid; q < nitems; q += 64) {
                const int vv = V.live[q / PRED_T], t = q - (q / PRED_T) * PRED_T;
                T ex, ey;
                pose_at(V.lanes, *V.rt, (int)V.lane[vv], V.ps0[vv], V.v[vv], V.rroad + vv * TTRL_ROUTE_MAX,
                        V.rlane + vv * TTRL_ROUTE_MAX, (int)V.rn[vv], t, ex, ey, (T*)nullptr);
                V.px[vv * PRED_T + t] = (float)ex;
                V.py[vv * PRED_T + t] = (float)ey;
              }
            }
            __syncthreads();
            PH(18);
            RG_INIT
            // is_conflict_possible (regulation.py:80-103) then respect_priorities (:62-77) for the pair
            // (a < b) of the env at LDS base ebp; a yield only ever sets ynew, so pairs commute
            auto reg_pair = [&](int ebp, int a, int b) {
              bool conflict = false;
              const int ka = ebp + a, kb = ebp + b;
              for (int t = 0; t < PRED_T && !conflict; ++t) {
                const int pa = ka * PRED_T + t, pb = kb * PRED_T + t;
                // float32 prefilter: a pair farther apart than LENGTH + the conversion and rounding
                // error bound (4e-7 of the coordinates' magnitude, 1 mm) is farther than LENGTH in
                // float64 too (NaN / inf fall through to the exact test)
                const float fxa = V.px[pa], fya = V.py[pa], fxb = V.px[pb], fyb = V.py[pb];
                const float fdx = fxb - fxa, fdy = fyb - fya;
                const float thr = float(P.length) + 1e-3f + 4e-7f * (fabsf(fxa) + fabsf(fxb) + fabsf(fya) + fabsf(fyb));
                if (fdx * fdx + fdy * fdy > thr * thr) continue;
                T xa, ya, ha, xb, yb, hb;  // the float64 poses, as predict_trajectory_constant_speed gives them
                pose_at(V.lanes, *V.rt, (int)V.lane[ka], V.ps0[ka], V.v[ka], V.rroad + ka * TTRL_ROUTE_MAX,
                        V.rlane + ka * TTRL_ROUTE_MAX, (int)V.rn[ka], t, xa, ya, &ha);
                pose_at(V.lanes, *V.rt, (int)V.lane[kb], V.ps0[kb], V.v[kb], V.rroad + kb * TTRL_ROUTE_MAX,
                        V.rlane + kb * TTRL_ROUTE_MAX, (int)V.rn[kb], t, xb, yb, &hb);
                const T dx = xb - xa, dy = yb - ya;
                if (sqrt(dx * dx + dy * dy) > T(P.length)) continue;
                conflict = rects_intersect(xa, ya, ha, xb, yb, hb, T(1.5) * T(P.length), T(0.9) * T(P.width));
              }
              if (!conflict) return;
              const int qa = V.lanes[V.lane[ebp + a]].prio, qb = V.lanes[V.lane[ebp + b]].prio;
              int yv;
              if (qa > qb) yv = b;
              else if (qa < qb) yv = a;
              else {
                const int ka = ebp + a, kb = ebp + b;
                const T fab = V.ch[ka] * (V.x[kb] - V.x[ka]) + V.sh[ka] * (V.y[kb] - V.y[ka]);
                const T fba = V.ch[kb] * (V.x[ka] - V.x[kb]) + V.sh[kb] * (V.y[ka] - V.y[kb]);
                yv = fab > fba ? a : b;
              }
              if (V.kind[ebp + yv] == TTRL_IDM) V.ynew[ebp + yv] = 1;  // ControlledVehicle, not MDPVehicle
            };
            if constexpr (NS * EPW == 64) {
              // One wavefront: the live pairs of the enforcing envs are spread over all its lanes
              // (a scene has ~8 live vehicles in 32 slots: slot-owned pairs left most lanes idle)
              const bool alive = V.kind[me] != TTRL_ABSENT;
              const unsigned long long am = __ballot(alive), dm = __ballot(doreg);
              constexpr unsigned long long SEG = NS == 64 ? ~0ull : ((1ull << NS) - 1);
              if (alive) V.live[eb + __popcll(((am >> eb) & SEG) & ((1ull << i) - 1))] = (uint8_t)i;
              int np[EPW], tot = 0;
#pragma unroll
              for (int e = 0; e < EPW; ++e) {
                const int n = ((dm >> (e * NS)) & 1ull) ? __popcll((am >> (e * NS)) & SEG) : 0;
                np[e] = n * (n - 1) / 2;
                tot += np[e];
              }
              __syncthreads();
              // pair k of the wave -> (env, lower live index, upper live index), pairs ordered by the upper
              auto decode = [&](int k, int& e, int& a, int& b) {
                int kk = k;
                e = 0;
                while (kk >= np[e]) { kk -= np[e]; ++e; }
                int rb = (int)((1.0f + sqrtf(1.0f + 8.0f * (float)kk)) * 0.5f);
                while (rb * (rb - 1) / 2 > kk) --rb;
                while ((rb + 1) * rb / 2 <= kk) ++rb;
                a = V.live[e * NS + kk - rb * (rb - 1) / 2];
                b = V.live[e * NS + rb];
              };
              // Flattened: is_conflict_possible is an OR over the 11 time steps, so (pair, step) items
              // are independent.  (P) a pair test: each vehicle's 11 predicted positions lie within its
              // reach of the middle one, so a pair whose middle positions are farther apart than both
              // reaches + the prefilter's threshold has no step that passes the prefilter (the triangle
              // inequality, with a rounding slack); the passing pairs are queued.  (A) the float32
              // distance prefilter over their (pair, step) items, survivors queued (ballot slots);
              // (B) the exact float64 test of the survivors, one per lane (a close pair no longer walks
              // its steps serially on one lane); (C) respect_priorities of the pairs that conflict.
              // The pairs run in chunks of RQ_PAIRS (a yield only sets ynew: chunks commute); an item
              // queue overflow takes the serial per-pair loop for its chunk.
              const float thr_len = float(P.length) + 1e-3f;
              float* reach = (float*)V.pd;  // [M], free until the projection; then the pair queue
              uint8_t* pq2 = (uint8_t*)V.pd + sizeof(float) * EPW * NS;  // [RQ_PAIRS] a chunk's passing pairs
              if (V.rq_cap > 0 && doreg && present) {
                const float* qx = V.px + me * PRED_T;
                const float* qy = V.py + me * PRED_T;
                const float cx = qx[PRED_T / 2], cy = qy[PRED_T / 2];
                float d2 = 0.0f;
                bool bad = false;  // a NaN position: the reach is unbounded
#pragma unroll
                for (int t = 0; t < PRED_T; ++t) {
                  const float dx = qx[t] - cx, dy = qy[t] - cy, dd = dx * dx + dy * dy;
                  bad |= dd != dd;
                  d2 = fmaxf(d2, dd);
                }
                reach[me] = bad ? INFINITY : sqrtf(d2);
              }
              if (tot > RQ_PAIRS) RG_COUNT(0);
              for (int c0 = 0; c0 < tot; c0 += RQ_PAIRS) {
                const int cn = tot - c0 < RQ_PAIRS ? tot - c0 : RQ_PAIRS;  // pairs c0 .. c0 + cn, ids k - c0
                bool flat = false;
                if (V.rq_cap > 0) {
                  for (int k = tid; k < cn; k += 64) V.rqf[k] = 0;
                  __syncthreads();
                  int np2 = 0;
                  for (int k0 = 0; k0 < cn; k0 += 64) {
                    const int k = k0 + tid;
                    bool pass = false;
                    if (k < cn) {
                      int e, a, b;
                      decode(c0 + k, e, a, b);
                      const int ka = e * NS + a, kb = e * NS + b;
                      const float cxa = V.px[ka * PRED_T + PRED_T / 2], cya = V.py[ka * PRED_T + PRED_T / 2];
                      const float cxb = V.px[kb * PRED_T + PRED_T / 2], cyb = V.py[kb * PRED_T + PRED_T / 2];
                      const float ra = reach[ka], rb = reach[kb];
                      const float dx = cxb - cxa, dy = cyb - cya;
                      // the prefilter's threshold at any step is at most thr_len + 4e-7 of the
                      // coordinates' magnitudes, each within its reach of the middle position; 1e-5
                      // relative + 1 cm cover the float32 rounding of this test, of the reaches and of
                      // the prefilter
                      const float thr =
                          thr_len + 4e-7f * (fabsf(cxa) + fabsf(cxb) + fabsf(cya) + fabsf(cyb) + 2.0f * (ra + rb));
                      const float bound = (ra + rb + thr) * 1.00001f + 1e-2f;
                      pass = !(dx * dx + dy * dy > bound * bound);  // NaN / inf pass
                    }
                    const unsigned long long bal = __ballot(pass);
                    if (pass) pq2[np2 + __popcll(bal & ((1ull << tid) - 1))] = (uint8_t)k;
                    np2 += __popcll(bal);
                  }
                  __syncthreads();
                  RG(0);
                  int nq = 0;
                  for (int k0 = 0; k0 < np2 * PRED_T; k0 += 64) {
                    const int k = k0 + tid;
                    bool pass = false;
                    int pid = 0, t = 0;
                    if (k < np2 * PRED_T) {
                      const int q = k / PRED_T;
                      t = k - q * PRED_T;
                      pid = pq2[q];
                      int e, a, b;
                      decode(c0 + pid, e, a, b);
                      const int ka = e * NS + a, kb = e * NS + b;
                      const int pa = ka * PRED_T + t, pb = kb * PRED_T + t;
                      const float fxa = V.px[pa], fya = V.py[pa], fxb = V.px[pb], fyb = V.py[pb];
                      const float fdx = fxb - fxa, fdy = fyb - fya;
                      const float thr = thr_len + 4e-7f * (fabsf(fxa) + fabsf(fxb) + fabsf(fya) + fabsf(fyb));
                      pass = !(fdx * fdx + fdy * fdy > thr * thr);  // as reg_pair's prefilter (NaN passes)
                    }
                    const unsigned long long bal = __ballot(pass);
                    const int pos = nq + __popcll(bal & ((1ull << tid) - 1));
                    if (pass && pos < V.rq_cap) V.rq[pos] = pid << 4 | t;
                    nq += __popcll(bal);
                  }
                  RG(1);
                  if (nq > V.rq_cap) RG_COUNT(1);
                  if (nq <= V.rq_cap) {
                    flat = true;
                    __syncthreads();
                    for (int k = tid; k < nq; k += 64) {
                      const int pid = V.rq[k] >> 4, t = V.rq[k] & 15;
                      int e, a, b;
                      decode(c0 + pid, e, a, b);
                      const int ka = e * NS + a, kb = e * NS + b;
                      T xa, ya, ha, xb, yb, hb;
                      pose_at(V.lanes, *V.rt, (int)V.lane[ka], V.ps0[ka], V.v[ka], V.rroad + ka * TTRL_ROUTE_MAX,
                              V.rlane + ka * TTRL_ROUTE_MAX, (int)V.rn[ka], t, xa, ya, &ha);
                      pose_at(V.lanes, *V.rt, (int)V.lane[kb], V.ps0[kb], V.v[kb], V.rroad + kb * TTRL_ROUTE_MAX,
                              V.rlane + kb * TTRL_ROUTE_MAX, (int)V.rn[kb], t, xb, yb, &hb);
                      const T dx = xb - xa, dy = yb - ya;
                      if (!(sqrt(dx * dx + dy * dy) > T(P.length)) &&
                          rects_intersect(xa, ya, ha, xb, yb, hb, T(1.5) * T(P.length), T(0.9) * T(P.width)))
                        V.rqf[pid] = 1;
                    }
                    __syncthreads();
                    RG(2);
                    for (int k = tid; k < cn; k += 64) {
                      if (!V.rqf[k]) continue;
                      int e, a, b;
                      decode(c0 + k, e, a, b);
                      const int ebp = e * NS;
                      const int qa = V.lanes[V.lane[ebp + a]].prio, qb = V.lanes[V.lane[ebp + b]].prio;
                      int yv;
                      if (qa > qb) yv = b;
                      else if (qa < qb) yv = a;
                      else {
                        const int ka = ebp + a, kb = ebp + b;
                        const T fab = V.ch[ka] * (V.x[kb] - V.x[ka]) + V.sh[ka] * (V.y[kb] - V.y[ka]);
                        const T fba = V.ch[kb] * (V.x[ka] - V.x[kb]) + V.sh[kb] * (V.y[ka] - V.y[kb]);
                        yv = fab > fba ? a : b;
                      }
                      if (V.kind[ebp + yv] == TTRL_IDM) V.ynew[ebp + yv] = 1;  // ControlledVehicle, not MDPVehicle
                    }
                  }
                }
                RG(3);
                if (!flat)
                  for (int k = tid; k < cn; k += 64) {
                    int e, a, b;
                    decode(c0 + k, e, a, b);
                    reg_pair(e * NS, a, b);
                  }
                RG(4);
                __syncthreads();  // the chunk's flags and queues read before the next chunk rewrites them
              }
            } else if (doreg) {  // every pair (a < b) once: thread i takes (i, i + d mod NS), d = 1 .. NS/2
              for (int d = 1; d <= NS / 2; ++d) {
                if (d == NS / 2 && i >= NS / 2) break;
                const int j = (i + d) & (NS - 1);
                const int a = i < j ? i : j, b = i < j ? j : i;
                if (V.kind[eb + a] == TTRL_ABSENT || V.kind[eb + b] == TTRL_ABSENT) continue;
                reg_pair(eb, a, b);
              }
            }
            __syncthreads();
            if (doreg && present && V.ynew[me]) {
              V.ts[me] = T(0);
              V.flags[me] |= FL_YIELD;
            }
          }
        }
      }
      PH(17);
      T x = V.x[me], y = V.y[me], h = V.h[me];
      if (present) {
        T v = V.v[me], steer = my_steer, acc = my_acc;
        int fl = V.flags[me];
        if (kind == TTRL_IDM) my_timer += dt;  // IDMVehicle.step behavior.py:147
        // Vehicle.clip_actions kinematics.py:155-168
        if (fl & FL_CRASHED) { steer = T(0); acc = T(-1) * v; }
        if (v > T(P.max_speed)) { const T c = T(1) * (T(P.max_speed) - v); if (c < acc) acc = c; }
        else if (v < T(P.min_speed)) { const T c = T(1) * (T(P.min_speed) - v); if (c > acc) acc = c; }
        my_steer = steer;
        my_acc = acc;
        // kinematic bicycle, Vehicle.step kinematics.py:140-153
        if (ablate & A_NO_KIN) {
          x += v * V.ch[me] * dt; y += v * V.sh[me] * dt; v += acc * dt;
        } else {
          // beta = atan(tan(steer) / 2) enters only through cos / sin of beta and of h + beta.
          // With (sd, cd) = sincos(steer), tan(beta) = sd / (2 cd), so cos(beta) =
          // 2 |cd| / sqrt(4 cd^2 + sd^2) and sin(beta) = sign(cd) sd / sqrt(4 cd^2 + sd^2); h + beta
          // by the angle sum on the resident cos / sin of h (a few ulp from the reference's direct
          // cos(h + beta), far inside the stated tolerances)
          const SinCos<T> sd = k_sincos(steer);
          const T inv = T(1) / sqrt(T(4) * (sd.c * sd.c) + sd.s * sd.s);
          const T cb = T(2) * fabs(sd.c) * inv, sb = (sd.c < T(0) ? -sd.s : sd.s) * inv;
          const T c0 = V.ch[me], s0 = V.sh[me];
          const T vx = v * (c0 * cb - s0 * sb), vy = v * (s0 * cb + c0 * sb);
          x += vx * dt; y += vy * dt;
          if (fl & FL_IMPACT) { x += my_ix; y += my_iy; fl = (fl | FL_CRASHED) & ~FL_IMPACT; }
          h += v * sb / (T(P.length) / T(2)) * dt;
          v += acc * dt;
          const SinCos<T> sc = k_sincos(h);
          V.ch[me] = sc.c; V.sh[me] = sc.s;
        }
        V.flags[me] = (uint8_t)fl;
        V.x[me] = x; V.y[me] = y; V.h[me] = h; V.v[me] = v;
        if constexpr (sizeof(T) == 8) V.xf[me] = (float)x;
      }
      PH(6);
      int cl;
      if constexpr (GR && NS * EPW == 64)
        cl = project_items<T, NS, EPW, LC>(V, P, nl, tid, le, i, present, !(ablate & A_NO_LANE), my_box, onb_all);
      else {
        int ob = 0;
        cl = project_all<T, NS, EPW, CV, !SO, LC>(V, P, nl, tid, le, i, present, x, y, h, !(ablate & A_NO_LANE), &ob);
        // this frame's order: the collision window below, the next frame's act
        if constexpr (SO && NS == 128) sort_order128<T>(V, nl, tid, false, my_sorted);
        else if constexpr (SO) sort_order<T, NS, EPW>(V, nl, tid, le, i, false, my_sorted, x, ob);
      }
      if (present && !(ablate & A_NO_LANE)) V.lane[me] = (int8_t)cl;  // on_state_update kinematics.py:170-177
      if (i == 0) V.pq_n[le] = 0;
      __syncthreads();
      PH(7);

      // collisions for all pairs (road.py:474-476, objects.py:91-137), impact: last writer.
      // Pass 1 (pipelined LDS loads): 1-D prefilter |dx| <= R, with R >= every pair's
      // threshold (diag + v*dt, v <= env max), so no pair the reference tests is dropped;
      // each lower-index vehicle then applies the reference's exact norm test to its pairs
      // (its own speed is the asymmetric threshold's) and queues the survivors.
      // Pass 2: the queued SATs run one pair per lane, each pair once.
      // Pass 3: every vehicle folds its pairs' results with the last-writer rule
      // (impact from the largest j > i that will intersect, else the largest i' < i).
      // A queue overflow (> NS pairs in an env) falls back to the per-vehicle sweep.
      const bool do_coll = !(ablate & A_NO_COLL);
      const T thr0 = (T(P.diagonal) + T(P.diagonal)) / T(2);
      // the pair (i, j > i) is tested against thr0 + v_i dt: i's own speed bounds its window
      const T Rw = thr0 + fabs(V.v[me]) * dt + T(1);
      constexpr int CH = NS < 64 ? NS : 64;
      if constexpr (NS <= 64) {
        // One wavefront: each vehicle i tests its partners j > i in a float window (its own speed
        // bounds the reference's asymmetric threshold), then the exact tests run one candidate per
        // lane per round, queue slots coming from the round's ballot (no LDS atomics).
        unsigned long long m = 0;
        if (SO && present && do_coll && V.stie[le] == 0) {
          // the window is a run of sorted positions (the float x is monotone in x): walk out from
          // this vehicle's position both ways while inside it
          const float xfi = V.xf[me];
          const float Rwf = (float)Rw * 1.0001f + 1e-5f * fabsf(xfi) + 1e-3f;
          const int p = V.spos[me];
          // WW positions each way per round, their LDS loads independent of each other (one LDS
          // latency per round instead of one per position; a window rarely spans more than WW)
          constexpr int WW = 3;
          int qu = p + 1, qd = p - 1;
          bool up = qu < NS, dn = qd >= 0;
          while (up || dn) {
            float xu[WW], xd[WW];
            int su[WW], sd[WW];
#pragma unroll
            for (int u = 0; u < WW; ++u) {
              const int a = min(qu + u, NS - 1), b = max(qd - u, 0);
              xu[u] = V.sxf[eb + a]; su[u] = V.sord[eb + a];
              xd[u] = V.sxf[eb + b]; sd[u] = V.sord[eb + b];
            }
#pragma unroll
            for (int u = 0; u < WW; ++u) {
              if (up) {
                if (qu + u < NS && !(xu[u] - xfi > Rwf)) m |= 1ull << su[u];
                else up = false;
              }
              if (dn) {
                if (qd - u >= 0 && !(xfi - xd[u] > Rwf)) m |= 1ull << sd[u];
                else dn = false;
              }
            }
            qu += WW;
            qd -= WW;
          }
          m &= ~((2ull << i) - 1);  // keep j > i
          if (ablate & A_NO_PREF) m = 0;
        } else if (present && do_coll) {
          const float xfi = V.xf[me];
          // float window: |xf_j - xf_i| in float errs by < 1.2e-7 (|x_i| + |x_j|), far below the slack
          const float Rwf = (float)Rw * 1.0001f + 1e-5f * fabsf(xfi) + 1e-3f;
#pragma unroll
          for (int j1 = 0; j1 < NS; j1 += 8) {
            float xs[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) xs[u] = V.xf[eb + j1 + u];
#pragma unroll
            for (int u = 0; u < 8; ++u)
              if (!(fabsf(xs[u] - xfi) > Rwf)) m |= 1ull << (j1 + u);
          }
          m &= ~((2ull << i) - 1);  // keep j > i
          if (ablate & A_NO_PREF) m = 0;
        }
        const T xi = V.x[me], yi = V.y[me], vi = V.v[me];
        const T thr = thr0 + vi * dt;
        // objects.py:123-133 exact, first for every window candidate (a few cheap rounds): norm >
        // thr drops the pair (far pairs skip it; inside thr - 1 no sqrt needed).  The 1-D window
        // also holds the vehicles of the other lanes at a similar x; dropping them here keeps the
        // expensive rounds below (one separating-axis proof per lane per round, the wave running
        // as many rounds as its busiest lane) to the pairs within the threshold.
        {
          unsigned long long mn = 0;
          for (unsigned long long mm = m; mm; mm &= mm - 1) {
            const int j = __ffsll((long long)mm) - 1;
            const T dx = V.x[eb + j] - xi, dy = V.y[eb + j] - yi;
            const T d2 = dx * dx + dy * dy;
            if (!(d2 > (thr + T(1)) * (thr + T(1))) &&
                !(!(thr > T(1) && d2 < (thr - T(1)) * (thr - T(1))) && sqrt(d2) > thr))
              mn |= 1ull << j;
          }
          m = mn;
        }
        const unsigned long long seg = NS == 64 ? ~0ull : ((1ull << NS) - 1) << ((tid & 63) / NS * NS);
        const unsigned long long below = (1ull << (tid & 63)) - 1;
        // The pairs within the threshold are queued first (cheap rounds, as many as the busiest
        // vehicle has pairs), then the separating-axis proofs run one pair per lane in a single
        // round, so a pile-up's vehicle with many close partners no longer serializes the proofs.
        // More close pairs than queue slots: pq_n > NS sends the env to pass 3's per-vehicle sweep.
        int base = 0;  // pairs of this env queued so far
        while (__any(m != 0)) {
          const bool has = m != 0;
          int j = 0;
          if (has) {
            j = __ffsll((long long)m) - 1;
            m &= m - 1;
          }
          const unsigned long long bal = __ballot(has) & seg;
          if (has) {
            const int q = base + __popcll(bal & below);
            if (q < NS) V.pq_ij[le * NS + q] = pair_pack(i, j, 0);
          }
          base += __popcll(bal);
        }
        if (base <= NS) {
          // the proofs, entry i on lane i; the survivors compacted in place (every lane reads its
          // entry before any lane writes)
          bool keep = false;
          int ij = 0;
          if (i < base) {
            ij = V.pq_ij[le * NS + i];
            const int a = eb + (ij & 0xff), b = eb + ((ij >> 8) & 0xff);
            // pairs the SAT provably separates contribute nothing
            keep = !sat_separated(P, V.x[a], V.y[a], V.ch[a], V.sh[a], V.v[a], V.x[b], V.y[b], V.ch[b], V.sh[b],
                                  V.v[b], dt);
          }
          const unsigned long long bal = __ballot(keep) & seg;
          if (keep) V.pq_ij[le * NS + __popcll(bal & below)] = ij;
          base = __popcll(bal);
        }
        if (i == 0) V.pq_n[le] = base;
      } else if (present && do_coll) {
        const T xi = V.x[me], yi = V.y[me], vi = V.v[me];
        const T thr = thr0 + vi * dt;
        // float window: |xf_j - xf_i| in float errs by < 1.2e-7 (|x_i| + |x_j|), far below the slack
        const float xfi = V.xf[me];
        const float Rwf = (float)Rw * 1.0001f + 1e-5f * fabsf(xfi) + 1e-3f;
        auto test_push = [&](int j) {
          const T dx = V.x[eb + j] - xi, dy = V.y[eb + j] - yi;
          const T d2 = dx * dx + dy * dy;
          if (d2 > (thr + T(1)) * (thr + T(1))) return;  // far: skip the exact test
          // objects.py:123-133 exact: norm > thr; inside thr - 1 it provably is not (no sqrt)
          if (!(thr > T(1) && d2 < (thr - T(1)) * (thr - T(1))) && sqrt(d2) > thr) return;
          if (sat_separated(P, xi, yi, V.ch[me], V.sh[me], vi, V.x[eb + j], V.y[eb + j], V.ch[eb + j], V.sh[eb + j],
                            V.v[eb + j], dt))
            return;  // provably (false, false): contributes nothing
          const int q = atomicAdd(&V.pq_n[le], 1);
          if (q < NS) V.pq_ij[le * NS + q] = pair_pack(i, j, 0);
        };
        if (SO && V.stie[le] == 0) {
          // the 128-slot sorted view: walk out from this vehicle's sorted position while inside the
          // window (the queue's order is free: pass 3 folds each vehicle's pairs by their indices),
          // keeping the partners within the exact norm threshold (cheap); the separating-axis
          // proofs then run over those only, so the wave's rounds follow its busiest lane's close
          // pairs rather than every vehicle of the other lanes at a similar x
          if (!(ablate & A_NO_PREF)) {
            constexpr int MW = (NS + 63) / 64;  // mask words (the sorted view: NS = 128)
            unsigned long long mk[MW];
#pragma unroll
            for (int w = 0; w < MW; ++w) mk[w] = 0ull;
            auto near = [&](int j) {
              const T dx = V.x[eb + j] - xi, dy = V.y[eb + j] - yi;
              const T d2 = dx * dx + dy * dy;
              if (d2 > (thr + T(1)) * (thr + T(1))) return;
              if (!(thr > T(1) && d2 < (thr - T(1)) * (thr - T(1))) && sqrt(d2) > thr) return;
              mk[j >> 6] |= 1ull << (j & 63);
            };
            const int p = V.spos[me];
            constexpr int WW = 3;  // positions each way per round, loaded independently (as NS <= 64)
            int qu = p + 1, qd = p - 1;
            bool up = qu < NS, dn = qd >= 0;
            while (up || dn) {
              float xu[WW], xd[WW];
              int su[WW], sd[WW];
#pragma unroll
              for (int u = 0; u < WW; ++u) {
                const int a = min(qu + u, NS - 1), b = max(qd - u, 0);
                xu[u] = V.sxf[eb + a]; su[u] = V.sord[eb + a];
                xd[u] = V.sxf[eb + b]; sd[u] = V.sord[eb + b];
              }
#pragma unroll
              for (int u = 0; u < WW; ++u) {
                if (up) {
                  if (qu + u < NS && !(xu[u] - xfi > Rwf)) {
                    if (su[u] > i) near(su[u]);
                  } else {
                    up = false;
                  }
                }
                if (dn) {
                  if (qd - u >= 0 && !(xfi - xd[u] > Rwf)) {
                    if (sd[u] > i) near(sd[u]);
                  } else {
                    dn = false;
                  }
                }
              }
              qu += WW;
              qd -= WW;
            }
#pragma unroll
            for (int w = 0; w < MW; ++w)
              for (unsigned long long mm = mk[w]; mm; mm &= mm - 1) {
                const int j = w * 64 + __ffsll((long long)mm) - 1;
                if (sat_separated(P, xi, yi, V.ch[me], V.sh[me], vi, V.x[eb + j], V.y[eb + j], V.ch[eb + j],
                                  V.sh[eb + j], V.v[eb + j], dt))
                  continue;  // provably (false, false): contributes nothing
                const int q = atomicAdd(&V.pq_n[le], 1);
                if (q < NS) V.pq_ij[le * NS + q] = pair_pack(i, j, 0);
              }
          }
        } else {
          // NS = 128: the slot index laundered, so the chunks' j > i masks and addresses are made
          // here (this is the rare tie path) rather than hoisted out of the frame loop and spilled
          int il = i, ebl = eb;
          if constexpr (NS > 64) asm volatile("" : "+v"(il), "+v"(ebl));
#pragma unroll
          for (int c0 = 0; c0 < NS; c0 += CH) {
            if (c0 + CH <= il + 1) continue;  // only partners j > i
            unsigned long long m = 0;
#pragma unroll
            for (int j1 = 0; j1 < CH; j1 += 8) {
              float xs[8];
#pragma unroll
              for (int u = 0; u < 8; ++u) xs[u] = V.xf[ebl + c0 + j1 + u];
#pragma unroll
              for (int u = 0; u < 8; ++u)
                if (!(fabsf(xs[u] - xfi) > Rwf)) m |= 1ull << (j1 + u);
            }
            if (il >= c0) m &= ~((2ull << (il - c0)) - 1);  // keep j > i
            if (ablate & A_NO_PREF) m = 0;
            while (m) {
              const int j = c0 + __ffsll((long long)m) - 1;
              m &= m - 1;
              test_push(j);
            }
          }
        }
      }
      __syncthreads();
      PH(8);
      const int npairs = do_coll ? V.pq_n[le] : 0;
      if (npairs <= NS && !(ablate & (A_NO_SAT | A_SAT_SERIAL))) {
        // Pass 2: 8 lanes per queued pair, one of the reference's 8 edge normals each (sat_axis),
        // combined in axis order: intersecting / will_intersect = no axis separates (ballot over
        // the lane group); translation = the first strict minimum of |distance| (min over the
        // group, ties to the lower axis), so the result equals sat_pair's.  Groups of 8 lanes
        // never straddle a wave or an env, and are either fully active or fully idle.
        int il = i;  // NS = 128: laundered, so the queue row's LDS address is not hoisted out of the
        if constexpr (NS > 64) asm volatile("" : "+v"(il));  // frame loop (and spilled to scratch)
        for (int t0 = 0; t0 < npairs * 8; t0 += NS) {
          const int t = t0 + il;
          if (t < npairs * 8) {
            const int q = t >> 3, kx = t & 7;
            const int ij = V.pq_ij[le * NS + q];
            const int a = eb + (ij & 0xff), b = eb + ((ij >> 8) & 0xff);
            T dd, dist, axx, axy;
            sat_axis(P, kx, V.x[a], V.y[a], V.ch[a], V.sh[a], V.v[a], V.x[b], V.y[b], V.ch[b], V.sh[b], V.v[b], dt,
                     dd, dist, axx, axy);
            const int g0 = (tid & 63) & ~7;
            const bool inter = ((__ballot(dd > T(0)) >> g0) & 0xffull) == 0;
            const bool will = ((__ballot(dist > T(0)) >> g0) & 0xffull) == 0;
            T bm = fabs(dist);
            if (bm != bm) bm = K<T>::inf();  // abs(nan) < min_distance is false: never chosen
            int bk = kx;
            auto merge = [&](T om, int ok, T ox, T oy) {
              if (om < bm || (om == bm && ok < bk)) { bm = om; bk = ok; axx = ox; axy = oy; }
            };
            merge(grp8_swap<1>(bm), grp8_swap<1>(bk), grp8_swap<1>(axx), grp8_swap<1>(axy));
            merge(grp8_swap<2>(bm), grp8_swap<2>(bk), grp8_swap<2>(axx), grp8_swap<2>(axy));
            merge(grp8_swap<4>(bm), grp8_swap<4>(bk), grp8_swap<4>(axx), grp8_swap<4>(axy));
            if (kx == 0) {
              V.pq_tx[le * NS + q] = will ? bm * axx : T(0);
              V.pq_ty[le * NS + q] = will ? bm * axy : T(0);
              V.pq_ij[le * NS + q] = pair_pack(ij & 0xff, (ij >> 8) & 0xff, (inter ? 1 : 0) | (will ? 2 : 0));
            }
          }
        }
      } else if (npairs <= NS && !(ablate & A_NO_SAT)) {
        for (int q = i; q < npairs; q += NS) {
          const int ij = V.pq_ij[le * NS + q], pi_ = ij & 0xff, pj_ = (ij >> 8) & 0xff;
          const int a = eb + pi_, b = eb + pj_;
          bool inter, will;
          T tx, ty;
          sat_pair(P, V.x[a], V.y[a], V.ch[a], V.sh[a], V.v[a], V.x[b], V.y[b], V.ch[b], V.sh[b], V.v[b], dt,
                   inter, will, tx, ty);
          V.pq_tx[le * NS + q] = tx;
          V.pq_ty[le * NS + q] = ty;
          V.pq_ij[le * NS + q] = pair_pack(pi_, pj_, (inter ? 1 : 0) | (will ? 2 : 0));
        }
      }
      __syncthreads();
      PH(9);
      if (present && do_coll && npairs > 0) {
        bool crash = false;
        int best_gt = -1, best_lt = -1;
        T gx = T(0), gy = T(0), lx = T(0), ly = T(0);
        if (npairs <= NS) {
          // the queue's row base, opaque to loop-invariant hoisting: hoisted out of the frame loop,
          // the three queue pointers were spilled to scratch (12 B per lane written back per launch)
          int qb = le * NS;
          asm volatile("" : "+v"(qb));
          for (int q = 0; q < npairs; ++q) {
            const int ij = V.pq_ij[qb + q], ri = ij & 0xff, rj = (ij >> 8) & 0xff, res = ij >> 16;
            if (ri == i) {
              if (res & 1) crash = true;
              if ((res & 2) && rj > best_gt) { best_gt = rj; gx = V.pq_tx[qb + q] / T(2); gy = V.pq_ty[qb + q] / T(2); }
            } else if (rj == i) {
              if (res & 1) crash = true;
              if ((res & 2) && ri > best_lt) { best_lt = ri; lx = -V.pq_tx[qb + q] / T(2); ly = -V.pq_ty[qb + q] / T(2); }
            }
          }
        } else {  // overflow: every vehicle sweeps all its partners in index order
          const T xi = V.x[me], yi = V.y[me], vi = V.v[me];
#pragma unroll 1
          for (int j = 0; j < NS; ++j) {
            if (j == i) continue;
            const T xj = V.x[eb + j], yj = V.y[eb + j], vj = V.v[eb + j];
            const bool lo = i < j;  // this vehicle is the reference's `self`
            if (fabs(xj - xi) > thr0 + fabs(lo ? vi : vj) * dt + T(1)) continue;
            const T dx = lo ? xj - xi : xi - xj, dy = lo ? yj - yi : yi - yj;
            const T thr = thr0 + (lo ? vi : vj) * dt;
            const T d2 = dx * dx + dy * dy;
            if (d2 > (thr + T(1)) * (thr + T(1))) continue;
            if (sqrt(d2) > thr) continue;
            const T ci = V.ch[me], si = V.sh[me], cj = V.ch[eb + j], sj = V.sh[eb + j];
            bool inter, will;
            T tx, ty;
            if constexpr (GR) {
              // the pair as the reference orders it (a = the lower index), one out-of-line call
              // returning by value: the road-network instance keeps it a call, and out-parameters
              // of a call would live in scratch
              const T ax = lo ? xi : xj, ay = lo ? yi : yj, ac = lo ? ci : cj, as = lo ? si : sj, av = lo ? vi : vj;
              const T bx = lo ? xj : xi, by = lo ? yj : yi, bc = lo ? cj : ci, bs = lo ? sj : si, bv = lo ? vj : vi;
              if (sat_separated(P, ax, ay, ac, as, av, bx, by, bc, bs, bv, dt)) continue;
              const SatRes<T> sr = sat_pair_v(P, ax, ay, ac, as, av, bx, by, bc, bs, bv, dt);
              inter = (sr.flags & 1) != 0; will = (sr.flags & 2) != 0; tx = sr.tx; ty = sr.ty;
            } else {  // inlined in both orders (the selected operands cost the straight instance a spill)
              if (lo ? sat_separated(P, xi, yi, ci, si, vi, xj, yj, cj, sj, vj, dt)
                     : sat_separated(P, xj, yj, cj, sj, vj, xi, yi, ci, si, vi, dt))
                continue;
              if (lo) sat_pair(P, xi, yi, ci, si, vi, xj, yj, cj, sj, vj, dt, inter, will, tx, ty);
              else sat_pair(P, xj, yj, cj, sj, vj, xi, yi, ci, si, vi, dt, inter, will, tx, ty);
            }
            if (will) {
              if (lo) { best_gt = j; gx = tx / T(2); gy = ty / T(2); }
              else { best_lt = j; lx = -tx / T(2); ly = -ty / T(2); }
            }
            if (inter) crash = true;
          }
        }
        int fl = V.flags[me];
        if (crash) fl |= FL_CRASHED;
        if (best_gt >= 0) { fl |= FL_IMPACT; my_ix = gx; my_iy = gy; }
        else if (best_lt >= 0) { fl |= FL_IMPACT; my_ix = lx; my_iy = ly; }
        V.flags[me] = (uint8_t)fl;
      }
    }
    PH(10);
  }
  __syncthreads();
  {
  // The thread's row indices and flags, re-derived from the (laundered) thread id after the frame
  // loop: kept live through the loop they were spilled to scratch, whose lines are written back
  // to HBM (~14 MB per 4096 x 64 launch).  The names shadow the prologue's.
  int tid_r = tid;
  asm volatile("" : "+v"(tid_r));
  const int le = tid_r / NS, i = tid_r % NS;
  const int env = env_at(ord, q0 + le, qend);
  const bool env_on = (unsigned)env < (unsigned)st.n_envs && (!env_mask || env_mask[env]);
  const bool slot = env_on && i < N;
  const size_t k = (size_t)env * N + i;
  const int me = le * NS + i;
  const int eb = le * NS;
  const int kind = V.kind[me];  // the view holds ABSENT for absent and out-of-range slots
  const bool present = kind != TTRL_ABSENT;
  if constexpr (EPI == EPI_IX) {
    ix_epilogue<T, NS, EPW>(V, st, R, P, so, *ie, le, i, env, env_on, slot, k, me, eb, reg, my_timer, my_steer.r,
                            my_acc.r, my_ix.r, my_iy.r, my_sidx);
  } else {
  if (slot) {  // LDS -> HBM, once per launch
    Veh<T> a;
    a.x = V.x[me]; a.y = V.y[me]; a.h = V.h[me]; a.v = V.v[me]; a.ts = V.ts[me]; a.timer = my_timer;
    a.steer = my_steer; a.acc = my_acc; a.ix = my_ix; a.iy = my_iy;
    a.lane = V.lane[me]; a.tgt = V.tgt[me]; a.sidx = PEEL ? 0 : my_sidx;  // PEEL: not stored, see the meta-action
    const int fl = V.flags[me];
    a.crashed = (fl & FL_CRASHED) != 0; a.hasimp = (fl & FL_IMPACT) != 0;
    if (!present) {  // absent rows pass through untouched
      a.x = ((const T*)st.x)[k]; a.lane = st.lane[k]; a.tgt = st.target_lane[k];
    }
    store_veh<!PEEL>(a, st, k);
    if constexpr (GR) {
      for (int q = 0; q < TTRL_ROUTE_MAX; ++q) {
        st.route_road[k * TTRL_ROUTE_MAX + q] = V.rroad[me * TTRL_ROUTE_MAX + q];
        st.route_lane[k * TTRL_ROUTE_MAX + q] = V.rlane[me * TTRL_ROUTE_MAX + q];
      }
      st.route_n[k] = V.rn[me];
      st.yielding[k] = (fl & FL_YIELD) ? 1 : 0;
    }
  }
  if constexpr (GR) {
    if (i == 0 && env_on) st.reg_steps[env] = reg;
  }
  PH(16);
  {
    // ttrl_env_step's tail, from LDS; scratch over the act phase's (dead) block (on a road network
    // that block also held the RegulatedRoad predictions, dead after the last frame as well)
    constexpr int M = EPW * NS;
    char* scr = (char*)V.afree;
    T* s_key = (T*)scr;
    int(*s_perm)[64] = (int(*)[64])(scr + ((sizeof(T) * M + 15) & ~(size_t)15));
    int(*s_p)[64] = s_perm + EPW;
    int* s_cnt = (int*)(s_p + EPW);
    int* s_ego = s_cnt + EPW;
    // the Kinematics observation of the final state (the 128-slot grid instance writes its grid
    // instead: compiled out there, its LDS row indices were spilled to scratch; at 64 slots the
    // register allocation came out worse without it, 0 -> 20 B per lane)
    if ((EPI != EPI_GRID || NS <= 64) && so.obs) {
      __syncthreads();
      auto ego_of = [&](int ego, T& ex, T& ey, T& eh, T& ev, T& ec, T& es, int& elane) {
        ex = V.x[eb + ego]; ey = V.y[eb + ego]; eh = V.h[eb + ego]; ev = V.v[eb + ego]; elane = V.lane[eb + ego];
        ec = V.ch[eb + ego]; es = V.sh[eb + ego];
      };
      kin_observe<T, NS, EPW>(st, V.lanes, P, so.kcfg, env_on, env, V.x[me], V.y[me], V.h[me], V.v[me], V.ch[me],
                              V.sh[me], (int)V.lane[me], present, present && kind == TTRL_MDP, ego_of, s_key, s_cnt,
                              s_ego, s_perm, s_p, so.obs, so.ids);
    }
    if (so.reward) {  // rewards_kernel's step tail (time += 1 / policy_frequency, rewards, dones, info)
      __syncthreads();
      if (i == 0) s_ego[le] = N;
      __syncthreads();
      if (present && kind == TTRL_MDP) atomicMin(&s_ego[le], i);
      __syncthreads();
      if (i == 0 && env_on) {
        const int ego = s_ego[le];
        step_tail<T>(R, V.lanes + (ego < N ? (int)V.lane[eb + ego] : 0), so.rcfg, env, ego < N, V.x[eb + ego % N], V.y[eb + ego % N], V.v[eb + ego % N],
                     (int)V.lane[eb + ego % N], (V.flags[eb + ego % N] & FL_CRASHED) != 0, V.v[eb],
                     (V.flags[eb] & FL_CRASHED) != 0, so.time, so.time_inc, so.reward, so.term, so.trunc, so.comp,
                     (T*)so.ego_speed, so.ego_crashed);
      }
    }
  }
  if constexpr (EPI == EPI_GRID) {  // the OccupancyGrid of the final state, from the view (EPW == 1)
    __syncthreads();  // its scratch overlays the tail's
    auto kind_of = [&](int j) { return (int)V.kind[eb + j]; };
    auto veh_of = [&](int j, T& vx, T& vy, T& vh, T& vv, T& vc, T& vs, int& vl) {
      vx = V.x[eb + j]; vy = V.y[eb + j]; vh = V.h[eb + j]; vv = V.v[eb + j]; vc = V.ch[eb + j]; vs = V.sh[eb + j];
      vl = V.lane[eb + j];
    };
    // the cfg is staged in LDS (word copies at constant offsets): indexed by feature in the loops,
    // the kernel argument itself would be copied to scratch
    constexpr int CW = sizeof(ttrl_grid_cfg_t) / 4;
    uint32_t* cw = (uint32_t*)(smem + ge->scr);
    if (i == 0) {
      const uint32_t* src = (const uint32_t*)&ge->cfg;
#pragma unroll
      for (int w = 0; w < CW; ++w) cw[w] = src[w];
    }
    __syncthreads();
    const ttrl_grid_cfg_t& gc = *(const ttrl_grid_cfg_t*)cw;
    if (env_on)
      grid_observe<T>(R, gc, N, i, NS, kind, V.x[me], V.y[me], V.h[me], V.v[me], V.ch[me], V.sh[me],
                      (int)V.lane[me], kind_of, veh_of,
                      grid_scratch<T>(smem + ge->scr + ((sizeof(ttrl_grid_cfg_t) + 15) & ~(size_t)15), gc, N),
                      ge->out + (size_t)env * ge->cfg.n_features * ge->cfg.shape_x * ge->cfg.shape_y,
                      TTRL_GRID_NT_STORES != 0);
  }
  }  // EPI != EPI_IX
  }
  PH_FLUSH
}

// Road.neighbour_vehicles for an explicit query lane per vehicle (road.py:480-513).
template <typename T, int NS, int EPW>
__global__ void __launch_bounds__(NS* EPW)
neighbours_kernel(ttrl_state_t st, ttrl_lane_table_t R, ttrl_params_t P, const int32_t* __restrict__ qlane,
                  int32_t* __restrict__ front, int32_t* __restrict__ rear) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, le = tid / NS, i = tid % NS;
  const int N = st.n_veh, nl = R.n_lanes;
  const int env = blockIdx.x * EPW + le;
  const bool slot = env < st.n_envs && i < N;
  const size_t k = (size_t)env * N + i;
  View<T> V = carve<T>(smem, EPW, NS, nl);
  stage_lanes(V, R, tid);
  T x = T(0), y = T(0);
  bool present = false;
  int l = 0;
  if (slot) {
    present = st.kind[k] != TTRL_ABSENT;
    x = ((const T*)st.x)[k];
    y = ((const T*)st.y)[k];
    l = qlane && qlane[k] >= 0 ? qlane[k] : st.lane[k];
    if (l < 0 || l >= nl) l = 0;
  }
  __syncthreads();
  project_all<T, NS, EPW>(V, P, nl, tid, le, i, present, x, y, T(0), false);
  __syncthreads();
  int ql[1] = {present ? l : -1};
  T s[1];
  T rr;
  lane_local(V.lanes[l], x, y, s[0], rr);
  int f[1], r[1];
  scan_neighbours<T, 1, NS, EPW>(V, le, i, ql, s, f, r);
  if (slot) { front[k] = f[0]; rear[k] = r[0]; }
}

// Vehicle.to_dict features (kinematics.py:237-261); route None => cos_d = sin_d = 0.
template <typename T>
__device__ __forceinline__ T feature(const LaneT<T>& L, int f, T x, T y, T h, T v, T c, T s) {
  switch (f) {
    case TTRL_F_PRESENCE: return T(1);
    case TTRL_F_X: return x;
    case TTRL_F_Y: return y;
    case TTRL_F_VX: return v * c;
    case TTRL_F_VY: return v * s;
    case TTRL_F_HEADING: return h;
    case TTRL_F_COS_H: return c;
    case TTRL_F_SIN_H: return s;
    case TTRL_F_LONG_OFF: case TTRL_F_LAT_OFF: case TTRL_F_ANG_OFF: {
      T ls, lr;
      lane_local(L, x, y, ls, lr);
      if (f == TTRL_F_LONG_OFF) return ls;
      if (f == TTRL_F_LAT_OFF) return lr;
      return wrap_to_pi(h - heading_at(L, ls));  // AbstractLane.local_angle lane.py:127-130
    }
    default: return T(0);
  }
}

// Philox4x32-10 (counter-based) for the "shuffled" row order.
// ------------------------------------------------------------ PCG64 (numpy) scene reset
struct U128 { unsigned long long hi, lo; };
__device__ __forceinline__ U128 mul128(U128 a, U128 b) {
  U128 r;
  r.lo = a.lo * b.lo;
  r.hi = __umul64hi(a.lo, b.lo) + a.hi * b.lo + a.lo * b.hi;
  return r;
}
__device__ __forceinline__ U128 add128(U128 a, U128 b) {
  U128 r;
  r.lo = a.lo + b.lo;
  r.hi = a.hi + b.hi + (r.lo < a.lo ? 1ull : 0ull);
  return r;
}
struct Pcg { U128 st, inc; bool has32; unsigned u32; };
__device__ __forceinline__ unsigned long long pcg_next64(Pcg& g) {
  const U128 M = {0x2360ED051FC65DA4ull, 0x4385DF649FCCF645ull};
  g.st = add128(mul128(g.st, M), g.inc);
  const unsigned long long x = g.st.hi ^ g.st.lo;
  const unsigned rot = (unsigned)(g.st.hi >> 58);
  return (x >> rot) | (x << ((64 - rot) & 63));
}
__device__ __forceinline__ unsigned pcg_next32(Pcg& g) {
  if (g.has32) { g.has32 = false; return g.u32; }
  const unsigned long long n = pcg_next64(g);
  g.has32 = true; g.u32 = (unsigned)(n >> 32);
  return (unsigned)n;
}
__device__ __forceinline__ double pcg_double(Pcg& g) {
  return (double)(pcg_next64(g) >> 11) * (1.0 / 9007199254740992.0);
}
__device__ __forceinline__ unsigned pcg_bounded(Pcg& g, unsigned n) {  // Generator.integers(0, n)
  if (n <= 1) return 0;
  const unsigned rng = n - 1;
  const unsigned long long rexcl = (unsigned long long)rng + 1;
  unsigned long long m = (unsigned long long)pcg_next32(g) * rexcl;
  unsigned left = (unsigned)m;
  if (left < rexcl) {
    const unsigned thr = (unsigned)((0xFFFFFFFFull - rng) % rexcl);
    while (left < thr) { m = (unsigned long long)pcg_next32(g) * rexcl; left = (unsigned)m; }
  }
  return (unsigned)(m >> 32);
}

// numpy.random.Generator over PCG64 (numpy random/src/distributions/distributions.c,
// _generator.pyx), the env's np_random (gymnasium seeding.np_random): state words
// {state_hi, state_lo, inc_hi, inc_lo, has_uint32 << 32 | uinteger} in ttrl_state_t.rng.
__device__ __forceinline__ Pcg rng_load(const uint64_t* w) {
  Pcg g;
  g.st = U128{w[0], w[1]};
  g.inc = U128{w[2], w[3]};
  g.has32 = (w[4] >> 32) != 0;
  g.u32 = (unsigned)w[4];
  return g;
}
__device__ __forceinline__ void rng_store(const Pcg& g, uint64_t* w) {
  w[0] = g.st.hi; w[1] = g.st.lo; w[2] = g.inc.hi; w[3] = g.inc.lo;
  w[4] = ((uint64_t)(g.has32 ? 1 : 0) << 32) | g.u32;
}
// random_interval: uniform on [0, max] by masked rejection (Generator.shuffle)
__device__ __forceinline__ unsigned pcg_interval(Pcg& g, unsigned max) {
  if (max == 0) return 0;
  unsigned mask = max;
  mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
  unsigned v;
  while ((v = (pcg_next32(g) & mask)) > max) {}
  return v;
}
#define TTRL_ZIG_QUAL __constant__
#include "ttrl_ziggurat.h"
// random_standard_normal: the 256-entry ziggurat of numpy (tables from gen_ziggurat.py)
__device__ __forceinline__ double pcg_normal_body(Pcg& g) {
  for (;;) {
    unsigned long long r = pcg_next64(g);
    const int idx = (int)(r & 0xff);
    r >>= 8;
    const int sign = (int)(r & 0x1);
    const unsigned long long rabs = (r >> 1) & 0x000fffffffffffffull;
    double x = (double)rabs * ttrl_zig_wi[idx];
    if (sign & 0x1) x = -x;
    if (rabs < ttrl_zig_ki[idx]) return x;
    if (idx == 0) {
      for (;;) {
        const double xx = -TTRL_ZIG_NOR_INV_R * log1p(-pcg_double(g));
        const double yy = -log1p(-pcg_double(g));
        if (yy + yy > xx * xx) return ((rabs >> 8) & 0x1) ? -(TTRL_ZIG_NOR_R + xx) : TTRL_ZIG_NOR_R + xx;
      }
    } else if (((ttrl_zig_fi[idx - 1] - ttrl_zig_fi[idx]) * pcg_double(g) + ttrl_zig_fi[idx]) < exp(-0.5 * x * x)) {
      return x;
    }
  }
}
// out of line in the scene kernels (one wavefront per env, many call sites); the simulate launch's
// fused spawn (ttrl_ix_env_step) inlines the body: a call there would give the road-network
// instance a stack
__device__ __noinline__ double pcg_normal(Pcg& g) { return pcg_normal_body(g); }
// Generator.choice(pop, size, replace=False), small population: Floyd's algorithm, then
// _shuffle_int (random_bounded_uint64 = buffered Lemire draws)
__device__ __forceinline__ void pcg_choice_noreplace(Pcg& g, int pop, int size, int* out) {
  for (int j = pop - size; j < pop; ++j) {
    const int val = (int)pcg_bounded(g, (unsigned)j + 1);
    bool seen = false;
    for (int q = 0; q < j - (pop - size); ++q) seen |= out[q] == val;
    out[j - (pop - size)] = seen ? j : val;
  }
  for (int i = size - 1; i >= 1; --i) {
    const int j = (int)pcg_bounded(g, (unsigned)i + 1);
    const int t = out[i]; out[i] = out[j]; out[j] = t;
  }
}

__device__ __forceinline__ uint4 philox(uint4 c, uint2 key) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const unsigned long long p0 = (unsigned long long)0xD2511F53u * c.x;
    const unsigned long long p1 = (unsigned long long)0xCD9E8D57u * c.z;
    c = make_uint4((unsigned)(p1 >> 32) ^ c.y ^ key.x, (unsigned)p1, (unsigned)(p0 >> 32) ^ c.w ^ key.y, (unsigned)p0);
    key.x += 0x9E3779B9u; key.y += 0xBB67AE85u;
  }
  return c;
}

// KinematicObservation.observe (observation.py:233-275): ego row + close_objects_to
// (road.py:418-447) stable-sorted by |lane distance| (or in list order when shuffled),
// normalised (lmap + clip), zero-padded.  The ego is the env's first MDP slot (AbstractEnv.vehicle).
// Shuffled: rows 1..V-1 permuted by np_random.shuffle(obs[1:]) (:272-273) with the env's own
// numpy Generator (order_shuffled 2, bit-exact) or by a Philox Fisher-Yates (1).
// Every thread of the workgroup calls it with its own vehicle's values (it synchronises the
// workgroup) -- hc, hs: cos / sin of its heading, k_sincos as the simulate kernel keeps them --
// and ego_of(ego, ex, ey, eh, ev, ec, es, elane) fetches the ego's.  The scratch arrays are
// s_key[EPW * NS], s_cnt[EPW], s_ego[EPW], s_perm[EPW][64], s_p[EPW][64].  Used by kinematics_obs_kernel and,
// fused after the last frame, by simulate_kernel (ttrl_env_step).
template <typename T, int NS, int EPW, typename EgoFn, typename PP>
__device__ __forceinline__ void kin_observe(const ttrl_state_t& st, const LaneT<T>* lanes, const PP& P,
                                            const ttrl_kin_cfg_t& cfg, bool env_ok, int env, T x, T y, T h, T v,
                                            T hc, T hs, int lane, bool present, bool mdp, EgoFn ego_of, T* s_key,
                                            int* s_cnt, int* s_ego, int (*s_perm)[64], int (*s_p)[64],
                                            float* __restrict__ out, int32_t* __restrict__ ids,
                                            float* __restrict__ out2, int32_t* __restrict__ ids2) {
  const int tid = threadIdx.x, le = tid / NS, i = tid % NS;
  const int N = st.n_veh;
  const bool slot = env_ok && i < N;
  if (i == 0) { s_cnt[le] = 0; s_ego[le] = NS; }
  __syncthreads();
  if (slot && mdp) atomicMin(&s_ego[le], i);
  __syncthreads();
  const int ego = s_ego[le];
  const bool has_ego = env_ok && ego < N;
  T ex = T(0), ey = T(0), eh = T(0), ev = T(0), ec = T(1), es = T(0);
  int elane = 0;
  if (has_ego) ego_of(ego, ex, ey, eh, ev, ec, es, elane);
  // candidate filter (road.py:427-433) and sort key |lane_distance_to| along the ego's lane
  bool cand = false;
  T key = K<T>::inf();
  if (has_ego && present && i != ego) {
    const T dx = x - ex, dy = y - ey;
    if (sqrt(dx * dx + dy * dy) < T(cfg.perception_distance)) {
      T s1, r1, s0, r0;
      lane_local(lanes[elane], x, y, s1, r1);
      lane_local(lanes[elane], ex, ey, s0, r0);
      const T ld = s1 - s0;
      if (cfg.see_behind || -T(2) * T(P.length) < ld) { cand = true; key = fabs(ld); }
    }
  }
  s_key[tid] = cand ? key : K<T>::nan();
  if (cand) atomicAdd(&s_cnt[le], 1);
  __syncthreads();
  int rank = 0;
  if (cand) {
    if (cfg.order_shuffled) {
      for (int j = 0; j < i; ++j) rank += s_key[le * NS + j] == s_key[le * NS + j] ? 1 : 0;
    } else {
      for (int j = 0; j < N; ++j) {
        const T kj = s_key[le * NS + j];
        rank += (kj < key || (kj == key && j < i)) ? 1 : 0;  // stable sort by key
      }
    }
  }
  int nc = env_ok ? s_cnt[le] : 0;
  const int V = cfg.vehicles_count, F = cfg.n_features;
  if (nc > V - 1) nc = V - 1;
  const bool shuf = cfg.order_shuffled && V - 1 <= 64;
  if (shuf) {
    if (i == 0 && env_ok) {
      int* p = s_p[le];  // in LDS: a private array would sit in scratch memory for every lane
      for (int t = 0; t < V - 1; ++t) p[t] = t;
      if (cfg.order_shuffled == 2) {  // Generator.shuffle: random_interval swaps, i = n-1 .. 1
        uint64_t* w = st.rng + (size_t)env * TTRL_RNG_WORDS;
        Pcg g = rng_load(w);
        for (int t = V - 2; t > 0; --t) {
          const int j = (int)pcg_interval(g, (unsigned)t);
          const int tmp = p[t]; p[t] = p[j]; p[j] = tmp;
        }
        rng_store(g, w);
      } else {  // Philox(seed, offset, env) Fisher-Yates: the multiset of rows is the reference's
        const uint2 key2 = make_uint2((unsigned)cfg.shuffle_seed, (unsigned)(cfg.shuffle_seed >> 32));
        for (int t = V - 2; t > 0; --t) {
          const uint4 r = philox(make_uint4((unsigned)env, (unsigned)t, (unsigned)cfg.shuffle_offset,
                                            (unsigned)(cfg.shuffle_offset >> 32)), key2);
          const int j = (int)(((unsigned long long)r.x * (unsigned)(t + 1)) >> 32);
          const int tmp = p[t]; p[t] = p[j]; p[j] = tmp;
        }
      }
      for (int t = 0; t < V - 1; ++t) s_perm[le][p[t]] = t;  // candidate row q -> output slot
    }
    __syncthreads();
  }
  if (!env_ok) return;
  // out2 / ids2 (this thread's env; ttrl_ix_env_step: an env that goes on keeps this observation as
  // the next step's): every row is written to both
  float* ob = out + (size_t)env * V * F;
  float* ob2 = out2 ? out2 + (size_t)env * V * F : nullptr;
  auto put = [&](int q, float val) {
    ob[q] = val;
    if (ob2) ob2[q] = val;
  };
  auto put_id = [&](int q, int32_t val) {
    if (ids) ids[(size_t)env * (V - 1) + q] = val;
    if (ids2) ids2[(size_t)env * (V - 1) + q] = val;
  };
  auto slot_of = [&](int q) { return shuf ? 1 + s_perm[le][q] : 1 + q; };
  auto emit = [&](int row, T px, T py, T phd, T pv, T c, T s, int pl, bool rel) {
    for (int cidx = 0; cidx < F; ++cidx) {
      const int f = cfg.features[cidx];
      T val = feature(lanes[pl], f, px, py, phd, pv, c, s);
      if (rel && !cfg.absolute && (f == TTRL_F_X || f == TTRL_F_Y || f == TTRL_F_VX || f == TTRL_F_VY))
        val -= feature(lanes[elane], f, ex, ey, eh, ev, ec, es);
      if (cfg.normalize && cfg.has_range[f]) {
        val = lmap(val, T(cfg.range_lo[f]), T(cfg.range_hi[f]), T(-1), T(1));
        if (cfg.clip) val = clip(val, T(-1), T(1));
      }
      put(row * F + cidx, (float)val);
    }
  };
  if (i == 0) {
    if (has_ego) emit(0, ex, ey, eh, ev, ec, es, elane, false);
    else for (int cidx = 0; cidx < F; ++cidx) put(cidx, 0.f);  // no controlled vehicle: zeros
  }
  if (cand && rank < nc) {
    emit(slot_of(rank), x, y, h, v, hc, hs, lane, true);
    put_id(rank, i);
  }
  for (int q = nc + i; q < V - 1; q += NS) {  // zero rows
    const int row = slot_of(q);
    for (int cidx = 0; cidx < F; ++cidx) put(row * F + cidx, 0.f);
    put_id(q, -1);
  }
}

// env_mask (optional): envs left untouched (rows and np_random) where it is 0.
template <typename T, int NS, int EPW>
__global__ void __launch_bounds__(NS* EPW)
kinematics_obs_kernel(ttrl_state_t st, ttrl_lane_table_t R, ttrl_params_t P, ttrl_kin_cfg_t cfg,
                      const uint8_t* __restrict__ env_mask, float* __restrict__ out, int32_t* __restrict__ ids) {
  __shared__ T s_key[EPW * NS];
  __shared__ int s_cnt[EPW], s_ego[EPW];
  __shared__ int s_perm[EPW][64], s_p[EPW][64];
  __shared__ LaneT<T> s_lanes[LMAX];
  const int tid = threadIdx.x, le = tid / NS, i = tid % NS;
  const int N = st.n_veh;
  const int env = blockIdx.x * EPW + le;
  const bool env_ok = env < st.n_envs && (!env_mask || env_mask[env]);
  const bool slot = env_ok && i < N;
  const size_t k = (size_t)env * N + i;
  if (tid < R.n_lanes) s_lanes[tid] = make_lane<T>(R, tid);
  T x = T(0), y = T(0), h = T(0), v = T(0);
  int lane = 0;
  bool present = false, mdp = false;
  if (slot) {
    x = ((const T*)st.x)[k]; y = ((const T*)st.y)[k]; h = ((const T*)st.heading)[k];
    v = ((const T*)st.speed)[k]; lane = st.lane[k];
    present = st.kind[k] != TTRL_ABSENT;
    mdp = st.kind[k] == TTRL_MDP;
  }
  auto ego_of = [&](int ego, T& ex, T& ey, T& eh, T& ev, T& ec, T& es, int& elane) {
    const size_t k0 = (size_t)env * N + ego;
    ex = ((const T*)st.x)[k0]; ey = ((const T*)st.y)[k0]; eh = ((const T*)st.heading)[k0];
    ev = ((const T*)st.speed)[k0]; elane = st.lane[k0];
    const SinCos<T> sc = k_sincos(eh);
    ec = sc.c; es = sc.s;
  };
  const SinCos<T> sc = k_sincos(h);
  kin_observe<T, NS, EPW>(st, s_lanes, P, cfg, env_ok, env, x, y, h, v, sc.c, sc.s, lane, present, mdp, ego_of, s_key,
                          s_cnt, s_ego, s_perm, s_p, out, ids);
}

// OccupancyGridObservation.observe (observation.py:353-434) + fill_road_layer_by_lanes
// (:453-483) of one env over the nt threads of a workgroup (grid_obs_kernel, and the fused
// env.step's epilogue, ttrl_env_step_grid).  The grid is assembled in LDS as per-cell winner
// vehicle indices (lowest list index wins = the reference's reverse-order overwrite) and streamed
// to HBM with 16-byte nontemporal stores.  Thread tid brings slot tid's vehicle in registers (kd
// TTRL_ABSENT if it has none); kind_of(j) / veh_of(j, x, y, h, v, cos, sin, lane) give any slot's.
template <typename T, typename KindOf, typename VehOf>
__device__ __forceinline__ void grid_observe(const ttrl_lane_table_t& R, const ttrl_grid_cfg_t& cfg, int N, int tid,
                                             int nt, int kd, T x, T y, T h, T v, T hc, T hs, int ln, KindOf kind_of,
                                             VehOf veh_of, const GridScr<T>& g, float* __restrict__ ob,
                                             bool nt_stores) {
  const int W = cfg.shape_x, H = cfg.shape_y, C = W * H, F = cfg.n_features;
  if (tid == 0) *g.ego = N;
  for (int c = tid; c < C; c += nt) g.win[c] = 0x7fffffff;
  for (int c = tid; c < (C + 31) / 32; c += nt) g.road[c] = 0u;
  __syncthreads();
  for (int j = tid; j < N; j += nt)
    if ((j == tid ? kd : kind_of(j)) == TTRL_MDP) atomicMin(g.ego, j);
  __syncthreads();
  // the observer: AbstractEnv.vehicle, the env's first MDP slot
  const int ego = *g.ego;
  if (ego >= N) {  // no controlled vehicle: an all-zero grid
    for (int q = tid; q < F * C; q += nt) __builtin_nontemporal_store(0.f, ob + q);
    return;
  }
  if (tid == ego % nt) {
    T ex, ey, eh, ev, ec, es;
    int el;
    if (ego == tid) { ex = x; ey = y; eh = h; ev = v; ec = hc; es = hs; el = ln; }
    else veh_of(ego, ex, ey, eh, ev, ec, es, el);
    g.e[0] = ex; g.e[1] = ey; g.e[2] = eh; g.e[3] = ev; g.e[4] = ec; g.e[5] = es; *g.elane = el;
  }
  __syncthreads();
  const T ex = g.e[0], ey = g.e[1], eh = g.e[2], ev = g.e[3], ec = g.e[4], es = g.e[5];
  const int elane = *g.elane;
  bool has_road = false;
  for (int c = 0; c < F; ++c) has_road |= cfg.features[c] == TTRL_F_ON_ROAD;
  const T rx0 = T(cfg.range_lo[TTRL_F_X]), rx1 = T(cfg.range_hi[TTRL_F_X]);
  const T ry0 = T(cfg.range_lo[TTRL_F_Y]), ry1 = T(cfg.range_hi[TTRL_F_Y]);
  const LaneT<T> EL = make_lane<T>(R, elane);
  for (int j = tid; j < N; j += nt) {
    T vx = x, vy = y, vh = h, vv = v, vc = hc, vs = hs;
    int vl = ln;
    if (j != tid) {  // slots beyond the block (N > nt)
      if (kind_of(j) == TTRL_ABSENT) continue;
      veh_of(j, vx, vy, vh, vv, vc, vs, vl);
    } else if (kd == TTRL_ABSENT) {
      continue;
    }
    const LaneT<T> L = make_lane<T>(R, vl);
    T rx = vx - ex, ry = vy - ey;
    for (int ci = 0; ci < F; ++ci) {
      const int f = cfg.features[ci];
      T val = feature(L, f, vx, vy, vh, vv, vc, vs);
      if (f == TTRL_F_X || f == TTRL_F_Y || f == TTRL_F_VX || f == TTRL_F_VY)
        val -= feature(EL, f, ex, ey, eh, ev, ec, es);
      if (cfg.has_range[f]) val = lmap(val, T(cfg.range_lo[f]), T(cfg.range_hi[f]), T(-1), T(1));
      if (cfg.clip) val = clip(val, T(-1), T(1));
      g.val[ci * N + j] = (float)val;
    }
    if (cfg.has_range[TTRL_F_X]) rx = lmap(lmap(rx, rx0, rx1, T(-1), T(1)), T(-1), T(1), rx0, rx1);
    if (cfg.has_range[TTRL_F_Y]) ry = lmap(lmap(ry, ry0, ry1, T(-1), T(1)), T(-1), T(1), ry0, ry1);
    const T fx = floor((rx - T(cfg.grid_min_x)) / T(cfg.step_x));
    const T fy = floor((ry - T(cfg.grid_min_y)) / T(cfg.step_y));
    if (T(0) <= fx && fx < T(W) && T(0) <= fy && fy < T(H)) atomicMin(&g.win[(int)fx * H + (int)fy], j);
  }
  if (has_road) {  // fill_road_layer_by_lanes observation.py:453-483, (lane, waypoint) items over the block
    const T spacing = T(cfg.step_x) < T(cfg.step_y) ? T(cfg.step_x) : T(cfg.step_y);
    const T lpd = T(cfg.lane_perception_distance);
    // items are handed out from the top of the block down, so the vehicle threads (the low ones)
    // take the fewest of them
    const int rt = nt - 1 - tid;
    long base = 0;
    for (int l = 0; l < R.n_lanes; ++l) {
      const LaneT<T> L = make_lane<T>(R, l);
      T origin, olat;
      lane_local(L, ex, ey, origin, olat);
      const T start = origin - lpd, stop = origin + lpd;
      const long n = (long)ceil((stop - start) / spacing);
      const T d1 = (start + spacing) - start;
      long q = ((rt - base) % nt + nt) % nt;  // this thread's first waypoint of the lane
      for (; q < n; q += nt) {
        T wp = q == 0 ? start : (q == 1 ? start + spacing : start + T(q) * d1);
        wp = clip(wp, T(0), T(R.length[l]));
        T px, py;
        lane_position(L, wp, T(0), px, py);
        px -= ex; py -= ey;
        const T fx = floor((px - T(cfg.grid_min_x)) / T(cfg.step_x));
        const T fy = floor((py - T(cfg.grid_min_y)) / T(cfg.step_y));
        if (T(0) <= fx && fx < T(W) && T(0) <= fy && fy < T(H)) {
          const int c = (int)fx * H + (int)fy;
          atomicOr(&g.road[c >> 5], 1u << (c & 31));
        }
      }
      base += n;
    }
  }
  __syncthreads();
  // the grid streams out once: 16-byte nontemporal stores (no reuse in L2); each thread owns
  // 4-cell groups and looks their winners up once for all feature layers.  !nt_stores: plain
  // stores (the fused launch's write-out, A/B)
  if ((C & 3) == 0) {
    typedef float f4 __attribute__((ext_vector_type(4)));
    for (int c4 = tid; c4 < C / 4; c4 += nt) {
      int w[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) w[u] = g.win[c4 * 4 + u];
      const unsigned rb = (g.road[c4 >> 3] >> ((c4 & 7) * 4)) & 0xfu;  // the 4 cells' on_road bits
      for (int ci = 0; ci < F; ++ci) {
        float r[4];
        if (cfg.features[ci] == TTRL_F_ON_ROAD) {
#pragma unroll
          for (int u = 0; u < 4; ++u) r[u] = ((rb >> u) & 1u) ? 1.f : 0.f;
        } else {
#pragma unroll
          for (int u = 0; u < 4; ++u) r[u] = w[u] == 0x7fffffff ? 0.f : g.val[ci * N + w[u]];
        }
        f4* dst = reinterpret_cast<f4*>(ob + (size_t)ci * C + c4 * 4);
        if (nt_stores) __builtin_nontemporal_store((f4){r[0], r[1], r[2], r[3]}, dst);
        else *dst = (f4){r[0], r[1], r[2], r[3]};
      }
    }
  } else {
    for (int ci = 0; ci < F; ++ci) {
      const bool road = cfg.features[ci] == TTRL_F_ON_ROAD;
      for (int c = tid; c < C; c += nt) {
        float r;
        if (road) r = ((g.road[c >> 5] >> (c & 31)) & 1u) ? 1.f : 0.f;
        else { const int w = g.win[c]; r = w == 0x7fffffff ? 0.f : g.val[ci * N + w]; }
        __builtin_nontemporal_store(r, ob + (size_t)ci * C + c);
      }
    }
  }
}

// One workgroup per env, one thread per slot (vehicles of slots beyond the block from HBM).
template <typename T>
__global__ void __launch_bounds__(256)
grid_obs_kernel(ttrl_state_t st, ttrl_lane_table_t R, ttrl_params_t P, ttrl_grid_cfg_t cfg, float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int env = blockIdx.x;
  const int N = st.n_veh;
  const size_t k0 = (size_t)env * N;
  // this thread's vehicle (slot tid; the block is sized so that normally every slot has one) is
  // loaded once, before the observer is known, so the block makes one HBM round trip
  const bool mine = tid < N;
  const size_t km = k0 + (mine ? tid : 0);
  const int kd = mine ? (int)st.kind[km] : TTRL_ABSENT;
  const T x = ((const T*)st.x)[km], y = ((const T*)st.y)[km], h = ((const T*)st.heading)[km];
  const T v = ((const T*)st.speed)[km];
  const int ln = st.lane[km];
  const SinCos<T> sc = t_sincos(h);
  auto kind_of = [&](int j) { return (int)st.kind[k0 + j]; };
  auto veh_of = [&](int j, T& vx, T& vy, T& vh, T& vv, T& vc, T& vs, int& vl) {
    const size_t k = k0 + j;
    vx = ((const T*)st.x)[k]; vy = ((const T*)st.y)[k]; vh = ((const T*)st.heading)[k]; vv = ((const T*)st.speed)[k];
    vl = st.lane[k];
    const SinCos<T> q = t_sincos(vh);
    vc = q.c; vs = q.s;
  };
  grid_observe<T>(R, cfg, N, tid, (int)blockDim.x, kd, x, y, h, v, sc.c, sc.s, ln, kind_of, veh_of,
                  grid_scratch<T>(smem, cfg, N), out + (size_t)env * cfg.n_features * cfg.shape_x * cfg.shape_y);
}

// ---------------------------------------------------------------------------------------
// TimeToCollisionObservation (observation.py:114-151) over compute_ttc_grid
// (finite_mdp.py:104-167).  One 64-thread workgroup per env, one lane per other vehicle;
// grid cells are `np.maximum` of costs {0.5, 1}, kept as OR-ed bits in LDS (bit0: 0.5 seen,
// bit1: 1 seen), so the list order of the reference's loop does not matter.
template <typename T>
__global__ void __launch_bounds__(64) ttc_obs_kernel(ttrl_state_t st, ttrl_lane_table_t R, ttrl_params_t P,
                                                     ttrl_ttc_cfg_t cfg, float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int* grid = (int*)smem;
  const int env = blockIdx.x, tid = threadIdx.x;
  const int N = st.n_veh, NS = P.n_target_speeds, NL = R.n_lanes, TB = cfg.horizon_bins;
  const size_t base = (size_t)env * N;
  for (int c = tid; c < NS * NL * TB; c += 64) grid[c] = 0;
  __syncthreads();
  const T* X = (const T*)st.x; const T* Y = (const T*)st.y; const T* H = (const T*)st.heading;
  const T* Vv = (const T*)st.speed;
  const int el = st.lane[base];
  const T ex = X[base], ey = Y[base];
  const T ec = t_cos(H[base]), es = t_sin(H[base]);
  const LaneT<T> EL = make_lane<T>(R, el);
  T s_ego, r_ego;
  lane_local(EL, ex, ey, s_ego, r_ego);
  for (int j = 1 + tid; j < N; j += 64) {
    if (st.kind[base + j] == TTRL_ABSENT) continue;
    const T vo = Vv[base + j];
    T s_o, r_o;
    lane_local(EL, X[base + j], Y[base + j], s_o, r_o);
    const T ld = s_o - s_ego;  // lane_distance_to objects.py:182-197
    const T proj = vo * (t_cos(H[base + j]) * ec + t_sin(H[base + j]) * es);
    const int lo = st.lane[base + j];
    const T margin = T(P.length) / T(2) + T(P.length) / T(2);
    for (int si = 0; si < NS; ++si) {
      const T ego_speed = T(P.target_speeds[si]);
      if (ego_speed == vo) continue;
      const T den = not_zero(ego_speed - proj);
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const T m = c == 0 ? T(0) : (c == 1 ? -margin : margin);
        const T ttc = (ld + m) / den;
        if (ttc < T(0)) continue;
        const T q = ttc / T(cfg.time_quantization);
        const T tq[2] = {q, ceil(q)};
#pragma unroll
        for (int u = 0; u < 2; ++u)
          if (tq[u] < T(TB)) atomicOr(&grid[(si * NL + lo) * TB + (int)tq[u]], c == 0 ? 2 : 1);
      }
    }
  }
  __syncthreads();
  if (cfg.obs_speeds == 0 && cfg.obs_lanes == 0) {  // the raw compute_ttc_grid (finite_mdp)
    float* ob = out + (size_t)env * NS * NL * TB;
    for (int k = tid; k < NS * NL * TB; k += 64) ob[k] = (grid[k] & 2) ? 1.0f : ((grid[k] & 1) ? 0.5f : 0.0f);
    return;
  }
  // observation.py:136-151: lane window padded with ones, speed rows repeated at the ends
  const int OS = cfg.obs_speeds, OL = cfg.obs_lanes, sidx = st.speed_index[base];
  float* ob = out + (size_t)env * OS * OL * TB;
  for (int k = tid; k < OS * OL * TB; k += 64) {
    const int a = k / (OL * TB), b = (k / TB) % OL, t = k % TB;
    const int row = NS + sidx - OS / 2 + a;
    const int sp = row < 1 + NS ? 0 : (row >= 2 * NS ? NS - 1 : row - NS);
    const int l = el - OL / 2 + b;
    float v = 1.0f;
    if (l >= 0 && l < NL) {
      const int g = grid[(sp * NL + l) * TB + t];
      v = (g & 2) ? 1.0f : ((g & 1) ? 0.5f : 0.0f);
    }
    ob[k] = v;
  }
}

// utils.distance_to_rect utils.py:386-413 (ray [r, q], rectangle corners c[0..3])
template <typename T>
__device__ __forceinline__ T ray_rect(T rx, T ry, T qx, T qy, const T (&c)[4][2]) {
  T ux = c[1][0] - c[0][0], uy = c[1][1] - c[0][1], vx = c[3][0] - c[0][0], vy = c[3][1] - c[0][1];
  const T nu = sqrt(ux * ux + uy * uy), nv = sqrt(vx * vx + vy * vy);
  ux /= nu; uy /= nu; vx /= nv; vy /= nv;
  const T qrx = qx - rx, qry = qy - ry;
  const T rqu = qrx * ux + qry * uy, rqv = qrx * vx + qry * vy;
  T a0 = ((c[0][0] - rx) * ux + (c[0][1] - ry) * uy) / rqu, a1 = ((c[1][0] - rx) * ux + (c[1][1] - ry) * uy) / rqu;
  T b0 = ((c[0][0] - rx) * vx + (c[0][1] - ry) * vy) / rqv, b1 = ((c[3][0] - rx) * vx + (c[3][1] - ry) * vy) / rqv;
  if (!(rqu >= T(0))) { const T t = a0; a0 = a1; a1 = t; }
  if (!(rqv >= T(0))) { const T t = b0; b0 = b1; b1 = t; }
  auto idist = [](T mina, T maxa, T minb, T maxb) { return mina < minb ? minb - maxa : mina - maxb; };
  if (idist(a0, a1, b0, b1) <= T(0) && idist(T(0), T(1), a0, a1) <= T(0) && idist(T(0), T(1), b0, b1) <= T(0))
    return (a0 > b0 ? a0 : b0) * sqrt(qrx * qrx + qry * qry);
  return K<T>::inf();
}

__device__ __forceinline__ unsigned long long ordered_bits(double d) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(d);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

// LidarObservation.trace (observation.py:704-752).  The reference updates a cell whenever a
// candidate's distance is <= the cell's current one, obstacle by obstacle in list order (its
// centre cell, then the cells its corners span): the final cell is the minimum distance, and
// among equal distances the last candidate in that order.  One workgroup per env, one lane per
// obstacle: pass 1 takes the LDS min of the ordered distance bits, pass 2 the max order among
// the candidates at that minimum, pass 3 lets that candidate write its relative speed.
template <typename T>
__global__ void __launch_bounds__(64) lidar_obs_kernel(ttrl_state_t st, ttrl_params_t P, ttrl_lidar_cfg_t cfg,
                                                       float* __restrict__ out) {
  __shared__ unsigned long long key[64];
  __shared__ int ord[64];
  __shared__ double dist[64], vel[64];
  const int env = blockIdx.x, tid = threadIdx.x;
  const int N = st.n_veh, C = cfg.cells;
  const size_t base = (size_t)env * N;
  const double range = cfg.maximum_range;
  const T step = T(2) * Tpi<T>() / T(C);
  if (tid < C) { key[tid] = ordered_bits(range); ord[tid] = -1; dist[tid] = range; vel[tid] = range; }
  __syncthreads();
  __shared__ int s_ego;  // the observer: the env's first MDP slot
  if (tid == 0) {
    int e = 0;
    while (e < N && st.kind[base + e] != TTRL_MDP) ++e;
    s_ego = e;
  }
  __syncthreads();
  const int ego = s_ego;
  if (ego >= N) {  // no controlled vehicle: maximum range everywhere
    for (int c = tid; c < C; c += 64) {
      out[((size_t)env * C + c) * 2] = (float)(cfg.normalize ? 1.0 : range);
      out[((size_t)env * C + c) * 2 + 1] = (float)(cfg.normalize ? 1.0 : range);
    }
    return;
  }
  const T* X = (const T*)st.x; const T* Y = (const T*)st.y; const T* H = (const T*)st.heading;
  const T* Vv = (const T*)st.speed;
  const size_t ke = base + ego;
  const T ox = X[ke], oy = Y[ke];
  const T ovx = Vv[ke] * t_cos(H[ke]), ovy = Vv[ke] * t_sin(H[ke]);
  auto to_index = [&](T a) {  // int(floor(a / step)) % cells, Python modulo
    long k = (long)floor(a / step) % C;
    return (int)(k < 0 ? k + C : k);
  };
  for (int pass = 0; pass < 3; ++pass) {
    for (int j = tid; j < N; j += 64) {
      if (j == ego || st.kind[base + j] == TTRL_ABSENT) continue;
      const T dx = X[base + j] - ox, dy = Y[base + j] - oy;
      const T center_distance = sqrt(dx * dx + dy * dy);
      if (center_distance > T(range)) continue;
      const T c = t_cos(H[base + j]), sn = t_sin(H[base + j]);
      const T vx = Vv[base + j] * c - ovx, vy = Vv[base + j] * sn - ovy;
      auto offer = [&](int cell, T d, int order) {
        if (d != d) return;  // NaN never satisfies distance <= grid
        const unsigned long long kb = ordered_bits((double)d);
        if (pass == 0) atomicMin(&key[cell], kb);
        else if (kb == key[cell]) {
          if (pass == 1) atomicMax(&ord[cell], order);
          else if (ord[cell] == order) {
            dist[cell] = (double)d;
            vel[cell] = (double)(vx * t_cos(T(cell) * step) + vy * t_sin(T(cell) * step));
          }
        }
      };
      offer(to_index(atan2(dy, dx) + step / T(2)), center_distance - T(P.width) / T(2), 2 * j);
      const T hl = T(P.length) / T(2), hw = T(P.width) / T(2);
      const T lc[4][2] = {{-hl, -hw}, {-hl, hw}, {hl, hw}, {hl, -hw}};
      T cr[4][2];
      T amin = T(0), amax = T(0);
#pragma unroll
      for (int q = 0; q < 4; ++q) {  // utils.rect_corners utils.py:126-155
        cr[q][0] = c * lc[q][0] + (-sn) * lc[q][1] + X[base + j];
        cr[q][1] = sn * lc[q][0] + c * lc[q][1] + Y[base + j];
        const T a = atan2(cr[q][1] - oy, cr[q][0] - ox) + step / T(2);
        if (q == 0 || a < amin) amin = a;
        if (q == 0 || a > amax) amax = a;
      }
      if (amin < -Tpi<T>() / T(2) && Tpi<T>() / T(2) < amax) {  // corners wrap around +pi
        const T t = amin;
        amin = amax;
        amax = t + T(2) * Tpi<T>();
      }
      const int start = to_index(amin), end = to_index(amax);
      const int n = start < end ? end - start + 1 : (C - start) + end + 1;
      for (int u = 0; u < n; ++u) {
        const int idx = start < end ? start + u : (u < C - start ? start + u : u - (C - start));
        const T dirx = t_cos(T(idx) * step), diry = t_sin(T(idx) * step);
        offer(idx, ray_rect(ox, oy, ox + T(range) * dirx, oy + T(range) * diry, cr), 2 * j + 1);
      }
    }
    __syncthreads();
  }
  if (tid < C) {  // observe(): obs /= maximum_range when normalize
    const double div = cfg.normalize ? range : 1.0;
    out[((size_t)env * C + tid) * 2] = (float)(dist[tid] / div);
    out[((size_t)env * C + tid) * 2 + 1] = (float)(vel[tid] / div);
  }
}

// numpy's SeedSequence(entropy words) -> generate_state(4, uint64) -> PCG64 seeding
// (numpy/random/bit_generator.pyx SeedSequence.mix_entropy / generate_state with pool_size 4,
// _pcg64.pyx + pcg64.h pcg64_set_seed: state = 0, inc = 2 * initseq + 1, step, state += seed,
// step).  Host and device, so np.random.default_rng([w0, w1, ...]) scenes can be generated on
// the GPU without a host round trip (device-side auto-reset) and the seeding tested on the CPU.
struct SeedSeq {
  static constexpr unsigned INIT_A = 0x43b0d7e5u, MULT_A = 0x931e8875u, INIT_B = 0x8b51f9ddu, MULT_B = 0x58f38dedu;
  static constexpr unsigned MIX_L = 0xca01f9ddu, MIX_R = 0x4973f715u;
  __host__ __device__ static unsigned hashmix(unsigned v, unsigned& h) {
    v ^= h;
    h *= MULT_A;
    v *= h;
    v ^= v >> 16;
    return v;
  }
  __host__ __device__ static unsigned mix(unsigned x, unsigned y) {
    unsigned r = MIX_L * x - MIX_R * y;
    r ^= r >> 16;
    return r;
  }
  // words: the entropy as uint32 words (numpy coerces each Python int < 2^32 to one word)
  __host__ __device__ static void pcg64_seed(const unsigned* words, int n, unsigned long long out[4]) {
    unsigned pool[4];
    unsigned h = INIT_A;
    for (int i = 0; i < 4; ++i) pool[i] = hashmix(i < n ? words[i] : 0u, h);
    for (int s = 0; s < 4; ++s)
      for (int d = 0; d < 4; ++d)
        if (s != d) pool[d] = mix(pool[d], hashmix(pool[s], h));
    for (int s = 4; s < n; ++s)
      for (int d = 0; d < 4; ++d) pool[d] = mix(pool[d], hashmix(words[s], h));
    unsigned st[8];
    unsigned hb = INIT_B;
    for (int i = 0; i < 8; ++i) {
      unsigned v = pool[i & 3];
      v ^= hb;
      hb *= MULT_B;
      v *= hb;
      v ^= v >> 16;
      st[i] = v;
    }
    unsigned long long w[4];
    for (int i = 0; i < 4; ++i) w[i] = (unsigned long long)st[2 * i] | ((unsigned long long)st[2 * i + 1] << 32);
    // pcg64_set_seed(seed = w[0] << 64 | w[1], inc = w[2] << 64 | w[3]), srandom_r
    const unsigned long long Mh = 0x2360ED051FC65DA4ull, Ml = 0x4385DF649FCCF645ull;
    unsigned long long inc_h = (w[2] << 1) | (w[3] >> 63), inc_l = (w[3] << 1) | 1ull;
    auto step = [&](unsigned long long& sh, unsigned long long& sl) {
      const unsigned long long lo = sl * Ml;
#ifdef __HIP_DEVICE_COMPILE__
      const unsigned long long hi = __umul64hi(sl, Ml) + sh * Ml + sl * Mh;
#else
      const unsigned long long hi = (unsigned long long)(((unsigned __int128)sl * Ml) >> 64) + sh * Ml + sl * Mh;
#endif
      sl = lo + inc_l;
      sh = hi + inc_h + (sl < lo ? 1ull : 0ull);
    };
    unsigned long long sh = 0, sl = 0;
    step(sh, sl);
    const unsigned long long ol = sl;
    sl += w[1];
    sh += w[0] + (sl < ol ? 1ull : 0ull);
    step(sh, sl);
    out[0] = sh; out[1] = sl; out[2] = inc_h; out[3] = inc_l;
  }
};

// RoadNetwork.get_closest_lane_index (road.py:55-71) in float64 over every lane, first minimum
// (CV = false: straight lanes along +x only, see lane_local).
template <bool CV = true>
__device__ inline int closest_lane_index(const ttrl_lane_table_t& R, double x, double y, double h) {
  int best = 0; double bd = 0;
  for (int l = 0; l < R.n_lanes; ++l) {
    const LaneT<double> L = make_lane<double>(R, l);
    double s, r;
    lane_local<CV>(L, x, y, s, r);
    const double ang = fabs(wrap_to_pi(h - heading_at<CV>(L, s)));
    double a = s - R.length[l]; if (!(a > 0)) a = 0;
    double c = 0 - s; if (!(c > 0)) c = 0;
    const double d = fabs(r) + a + c + 1.0 * ang;
    if (l == 0 || d < bd) { bd = d; best = l; }
  }
  return best;
}

// Scene generation: ego MDPVehicle, then n-1 x IDMVehicle.create_random
// (kinematics.py:50-104) + randomize_behavior (behavior.py:66-69), the numpy RNG stream
// reproduced bit for bit, one env in draw order.
template <typename T, typename PP>
__device__ void reset_env_serial(const ttrl_state_t& st, const ttrl_lane_table_t& R, const PP& P,
                                 const ttrl_reset_cfg_t& cfg, Pcg g, int env) {
  const int N = st.n_veh, nl = R.n_lanes;
  const size_t b = (size_t)env * N;
  T* X = (T*)st.x; T* Y = (T*)st.y; T* Hh = (T*)st.heading; T* Vv = (T*)st.speed; T* TS = (T*)st.target_speed;
  T* TM = (T*)st.timer; T* DL = (T*)st.delta;
  double smax[LMAX];
  auto track = [&](double x, double y, bool first) {
    for (int l = 0; l < nl; ++l) {
      double s, r;
      lane_local(make_lane<double>(R, l), x, y, s, r);
      if (first || s > smax[l]) smax[l] = s;
    }
  };
  for (int i = 0; i < N; ++i) {
    const size_t k = b + i;
    st.kind[k] = TTRL_ABSENT; st.crashed[k] = 0; st.has_impact[k] = 0; st.lane_change[k] = 0;
    X[k] = Y[k] = Hh[k] = Vv[k] = TS[k] = TM[k] = T(0);
    ((T*)st.steer)[k] = ((T*)st.acc)[k] = ((T*)st.impact_x)[k] = ((T*)st.impact_y)[k] = T(0);
    DL[k] = T(4); st.lane[k] = st.target_lane[k] = 0; st.speed_index[k] = -1;
  }
  {
    const int l = cfg.ego_lane;
    const LaneT<double> L = make_lane<double>(R, l);
    double ex, ey;
    lane_position(L, cfg.ego_x, 0.0, ex, ey);
    const double eh = heading_at(L, cfg.ego_x);
    st.kind[b] = TTRL_MDP; X[b] = T(ex); Y[b] = T(ey); Hh[b] = T(eh); Vv[b] = T(cfg.ego_speed);
    const int ln = closest_lane_index(R, ex, ey, eh);
    st.lane[b] = st.target_lane[b] = ln;
    const int si = speed_to_index(P, cfg.ego_speed);
    st.speed_index[b] = si;
    TS[b] = T(P.target_speeds[si]);
    track(ex, ey, true);
  }
  for (int i = 1; i < cfg.n_vehicles && i < N; ++i) {
    const size_t k = b + i;
    const int lid = (int)pcg_bounded(g, (unsigned)nl);
    const double sp = cfg.speed_lo + (cfg.speed_hi - cfg.speed_lo) * pcg_double(g);
    const double offset = cfg.spacing * (12 + 1.0 * sp) * cfg.density_factor;
    double x0 = smax[lid];
    x0 += offset * (0.9 + (1.1 - 0.9) * pcg_double(g));
    const LaneT<double> L = make_lane<double>(R, lid);
    double px, py;
    lane_position(L, x0, 0.0, px, py);
    const double ph = heading_at(L, x0);
    st.kind[k] = TTRL_IDM; st.lane_change[k] = (uint8_t)cfg.lane_change;
    X[k] = T(px); Y[k] = T(py); Hh[k] = T(ph); Vv[k] = T(sp); TS[k] = T(sp);
    const int ln = closest_lane_index(R, px, py, ph);
    st.lane[k] = st.target_lane[k] = ln;
    TM[k] = T(pymod((px + py) * 3.141592653589793, P.lane_change_delay));
    DL[k] = T(cfg.delta_lo + (cfg.delta_hi - cfg.delta_lo) * pcg_double(g));
    track(px, py, false);
  }
}

// A double of lane `l` (wave-uniform index) of the wavefront, as a uniform value.
__device__ __forceinline__ double readlane_d(double v, int l) {
  const long long b = __double_as_longlong(v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)b, l);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

__device__ __forceinline__ unsigned long long shfl_u64(unsigned long long v, int src) {
  const unsigned lo = (unsigned)__shfl((int)(unsigned)v, src & 63, 64);
  const unsigned hi = (unsigned)__shfl((int)(unsigned)(v >> 32), src & 63, 64);
  return ((unsigned long long)hi << 32) | lo;
}
__device__ __forceinline__ double shfl_d(double v, int src) {
  return __longlong_as_double((long long)shfl_u64((unsigned long long)__double_as_longlong(v), src));
}

__device__ __forceinline__ unsigned long long pcg_output(U128 st) {  // pcg_next64's output of a state
  const unsigned long long x = st.hi ^ st.lo;
  const unsigned rot = (unsigned)(st.hi >> 58);
  return (x >> rot) | (x << ((64 - rot) & 63));
}
__device__ __forceinline__ double pcg_unit(unsigned long long o) {
  return (double)(o >> 11) * (1.0 / 9007199254740992.0);
}

// The same scene as reset_env_serial, one wavefront per env (lane = vehicle slot), for the masked
// auto-reset on the critical path of env.step.  numpy's draw order is sequential, but its stream
// is not: vehicle i (1-based) consumes the 64-bit outputs from index c(i) = 3 (i - 1) + i / 2 on
// (odd i: one output for integers(0, lanes) -- its high half buffered -- and three for the
// uniforms; even i: the buffered half, then three).  The LCG step s -> M s + inc is affine, so a
// scan of the vehicles' k-step maps (M^k, 1 + M + .. + M^(k-1)) over the wavefront gives every lane
// its generator state at c(i) (numpy pcg64_advance, in parallel), and each lane draws its
// vehicle's lane, speed, gap and DELTA.  Only the placement is a recurrence (x0 = the max s on the
// drawn lane so far + the gap): it runs wave-uniformly with reset_env_serial's exact arithmetic --
// on the highway (straight +x lanes from one start x) as one chain of float64 adds -- then every
// lane assigns its vehicle's pose, lane and timer and the rows are written coalesced.  A Lemire rejection in
// integers() (probability < 2^-31 per draw, never for a power-of-two lane count) would shift the
// stream: such an env is regenerated by the sequential replay (reset_env_serial).
// AutoReset: the env.step auto-reset bookkeeping folded into the reset launch (ttrl_auto_reset_highway):
// done = terminated | truncated, written to done_out; a done env bumps its entropy word `ep_word`
// (the episode counter), seeds from the bumped words and gets time = 0.
struct AutoReset {
  const uint8_t* term;
  const uint8_t* trunc;
  double* time;
  uint8_t* done_out;
  int ep_word;
};

template <typename T, bool CV>
__global__ void __launch_bounds__(64) reset_wave_kernel(ttrl_state_t st, ttrl_lane_table_t R, ttrl_params_t P,
                                                        ttrl_reset_cfg_t cfg, const unsigned long long* __restrict__ pcg,
                                                        unsigned* __restrict__ words, int n_words,
                                                        const uint8_t* __restrict__ mask, AutoReset ar) {
  const int env = blockIdx.x, lane = threadIdx.x;
  if (env >= st.n_envs) return;
  if (ar.term) {  // auto-reset: the done mask, episode counter and time in the same launch
    const bool done = ar.term[env] || ar.trunc[env];
    if (lane == 0) ar.done_out[env] = (uint8_t)done;
    if (!done) return;
  } else if (mask && !mask[env]) {
    return;
  }
#ifdef TTRL_RESET_TRACE  // -DTTRL_RESET_TRACE: phase clocks of a few envs (tools/reset_phases.py)
  long long tr[8];
  int ntr = 0;
#define RT() tr[ntr++] = wall_clock64()
  RT();
#else
#define RT()
#endif
  const int N = st.n_veh, nl = R.n_lanes, nv = min(cfg.n_vehicles, N);
  const size_t b = (size_t)env * N;
  T* X = (T*)st.x; T* Y = (T*)st.y; T* Hh = (T*)st.heading; T* Vv = (T*)st.speed; T* TS = (T*)st.target_speed;
  T* TM = (T*)st.timer; T* DL = (T*)st.delta;
  unsigned long long s4[4];
  if (pcg) {
    for (int k = 0; k < 4; ++k) s4[k] = pcg[4 * env + k];
  } else if (ar.term) {  // (n_words <= 8; the bumped word picked by selects: no scratch array)
    unsigned w[8];
#pragma unroll
    for (int q = 0; q < 8; ++q)
      w[q] = q < n_words ? words[(size_t)env * n_words + q] + (q == ar.ep_word ? 1u : 0u) : 0u;
    SeedSeq::pcg64_seed(w, n_words, s4);
    if (lane == 0) {
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (q == ar.ep_word) words[(size_t)env * n_words + q] = w[q];
      ar.time[env] = 0.0;
    }
  } else {
    SeedSeq::pcg64_seed(words + (size_t)env * n_words, n_words, s4);
  }
  const U128 s0 = {s4[0], s4[1]}, inc = {s4[2], s4[3]};
  RT();
  // lane k < nl keeps lane k's geometry and the max s on lane k of the vehicles placed so far
  LaneT<double> myL;
  if (lane < nl) myL = make_lane<double>(R, lane);
  double my_smax = 0;
  // the ego MDPVehicle (slot 0)
  double ex = 0, ey = 0, eh = 0;
  {
    const LaneT<double> L = make_lane<double>(R, cfg.ego_lane);
    lane_position(L, cfg.ego_x, 0.0, ex, ey);
    eh = heading_at(L, cfg.ego_x);
    if (lane < nl) {
      double s, r;
      lane_local<CV>(myL, ex, ey, s, r);
      my_smax = s;
    }
  }
  // straight +x lanes from one start x (the highway): one running max of s for every lane
  const double sx0 = readlane_d(myL.sx, 0);
  const bool same_start = !CV && !__any(lane < nl && myL.sx != sx0);
  double run_max = readlane_d(my_smax, 0);
  const unsigned rng_ = (unsigned)nl - 1;
  const unsigned long long rexcl = (unsigned long long)rng_ + 1;
  const unsigned thr = nl > 1 ? (unsigned)((0xFFFFFFFFull - rng_) % rexcl) : 0u;
  unsigned carry_hi = 0;  // the buffered half of the previous chunk's last (odd) vehicle
  U128 chunk_state = s0, next_state = s0;  // the LCG state at the chunk's first draw
  bool reject = false;
  for (int c0 = 0; c0 < N; c0 += 64) {
    const int i = c0 + lane;
    const bool drawn = i >= 1 && i < nv;
    // ---- parallel draws (lane = vehicle i)
    double sp = 0, d = 0, delta = 0;
    int lid = 0;
    unsigned u32 = 0, hi32 = 0;
    unsigned long long o1 = 0, o2 = 0, o3 = 0;
    {
      // the LCG state before vehicle i: the chunk's start state advanced by the exclusive prefix of
      // the vehicles' output counts (4 odd, 3 even, 0 the ego), as a scan of affine maps
      // s -> A s + C inc over the wave (A, C: powers and partial sums of the multiplier)
      const int len = drawn ? ((i & 1) ? 4 : 3) : 0;
      U128 A = {0ull, 1ull}, Cs = {0ull, 0ull};  // identity
      // M^3, 1 + M + M^2 and M^4, 1 + M + M^2 + M^3 (mod 2^128), M the PCG64 multiplier
      if (len == 3) { A = {0x25f041404bd80e82ull, 0xeb5ae837ed42153dull}; Cs = {0x3b1dd060ff2fd1e0ull, 0x9624b94fc0ada4dfull}; }
      if (len == 4) { A = {0xf4dd417327db7a9bull, 0xd194dfbe42d45771ull}; Cs = {0x610e11a14b07e063ull, 0x817fa187adefba1cull}; }
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {  // inclusive scan: (A, Cs) <- own o earlier
        U128 Ap, Cp;
        Ap.hi = shfl_u64(A.hi, lane - off); Ap.lo = shfl_u64(A.lo, lane - off);
        Cp.hi = shfl_u64(Cs.hi, lane - off); Cp.lo = shfl_u64(Cs.lo, lane - off);
        if (lane >= off) {
          Cs = add128(mul128(A, Cp), Cs);
          A = mul128(A, Ap);
        }
      }
      // exclusive: the maps of the lanes below; the chunk's start state from the carry
      U128 Ae, Ce;
      Ae.hi = shfl_u64(A.hi, lane - 1); Ae.lo = shfl_u64(A.lo, lane - 1);
      Ce.hi = shfl_u64(Cs.hi, lane - 1); Ce.lo = shfl_u64(Cs.lo, lane - 1);
      if (lane == 0) { Ae = {0ull, 1ull}; Ce = {0ull, 0ull}; }
      U128 g = add128(mul128(Ae, chunk_state), mul128(Ce, inc));
      U128 An, Cn;  // the whole chunk (lane 63's inclusive map): the next chunk's start state
      An.hi = shfl_u64(A.hi, 63); An.lo = shfl_u64(A.lo, 63);
      Cn.hi = shfl_u64(Cs.hi, 63); Cn.lo = shfl_u64(Cs.lo, 63);
      next_state = add128(mul128(An, chunk_state), mul128(Cn, inc));
      if (drawn) {
        const U128 M = {0x2360ED051FC65DA4ull, 0x4385DF649FCCF645ull};
        if (i & 1) {  // integers(0, lanes) draws a fresh output: low half now, high half buffered
          g = add128(mul128(g, M), inc);
          const unsigned long long o = pcg_output(g);
          u32 = (unsigned)o;
          hi32 = (unsigned)(o >> 32);
        }
        g = add128(mul128(g, M), inc); o1 = pcg_output(g);
        g = add128(mul128(g, M), inc); o2 = pcg_output(g);
        g = add128(mul128(g, M), inc); o3 = pcg_output(g);
      }
    }
    // even vehicles take the previous (odd) vehicle's buffered half: lane - 1, or the carry
    const unsigned prev_hi = (unsigned)__shfl((int)hi32, (lane + 63) & 63, 64);
    if (drawn) {
      if (!(i & 1)) u32 = lane == 0 ? carry_hi : prev_hi;
      if (nl > 1) {
        const unsigned long long m = (unsigned long long)u32 * rexcl;
        if ((unsigned)m < thr) reject = true;
        lid = (int)(m >> 32);
      }
      sp = cfg.speed_lo + (cfg.speed_hi - cfg.speed_lo) * pcg_unit(o1);
      const double offset = cfg.spacing * (12 + 1.0 * sp) * cfg.density_factor;
      d = offset * (0.9 + (1.1 - 0.9) * pcg_unit(o2));
      delta = cfg.delta_lo + (cfg.delta_hi - cfg.delta_lo) * pcg_unit(o3);
    }
    carry_hi = (unsigned)__shfl((int)hi32, 63, 64);
    chunk_state = next_state;
    if (c0 == 0) RT();
    // ---- the placement recurrence, in draw order: x0 = (max s on the drawn lane) + gap; the
    // vehicle's pose is computed wave-uniformly, then every lane k < nl folds its own s into its max
    double px = 0, py = 0, ph = 0;
    const int n = min(64, nv - c0);
    if (!CV && same_start) {
      // every lane straight along +x from one start x: a vehicle's s is the same on every lane, so
      // the per-lane maxima are one running max and the recurrence is a chain of float64 adds
      // (the same operations as the general path, hence the same bits)
      double x0_own = 0;
      for (int q = c0 == 0 ? 1 : 0; q < n; ++q) {
        double x0 = run_max;
        x0 += readlane_d(d, q);
        const double qx = sx0 + x0 * 1.0 + 0.0 * (-0.0);  // lane_position_straight's x
        const double sq = qx - sx0;                        // lane_local's s
        if (sq > run_max) run_max = sq;
        if (lane == q) x0_own = x0;
      }
      // the pose on the drawn lane, from that lane's geometry (shuffles with every lane active:
      // a bpermute from an inactive lane returns 0)
      LaneT<double> L = {};
      L.sx = shfl_d(myL.sx, lid); L.sy = shfl_d(myL.sy, lid);
      L.dx = shfl_d(myL.dx, lid); L.dy = shfl_d(myL.dy, lid);
      L.hd = shfl_d(myL.hd, lid);
      if (i < nv && i >= 1) {
        lane_position_straight(L, x0_own, 0.0, px, py);
        ph = L.hd;
      }
    } else {
      for (int q = c0 == 0 ? 1 : 0; q < n; ++q) {
        const int lq = __builtin_amdgcn_readlane(lid, q);
        double x0 = readlane_d(my_smax, lq);
        x0 += readlane_d(d, q);
        double qx, qy, qh;
        if constexpr (!CV) {  // straight +x lanes: the drawn lane's geometry from the lane holding it
          LaneT<double> L = {};
          L.type = TTRL_LANE_STRAIGHT;
          L.sx = readlane_d(myL.sx, lq); L.sy = readlane_d(myL.sy, lq);
          L.dx = readlane_d(myL.dx, lq); L.dy = readlane_d(myL.dy, lq);
          L.hd = readlane_d(myL.hd, lq);
          lane_position_straight(L, x0, 0.0, qx, qy);
          qh = L.hd;
        } else {
          const LaneT<double> L = make_lane<double>(R, lq);
          lane_position(L, x0, 0.0, qx, qy);
          qh = heading_at(L, x0);
        }
        if (lane == q) { px = qx; py = qy; ph = qh; }
        if (lane < nl) {
          double s, r;
          lane_local<CV>(myL, qx, qy, s, r);
          if (s > my_smax) my_smax = s;
        }
      }
    }
    if (c0 == 0) RT();
    // ---- every slot of the chunk, coalesced
    if (i < N) {
      const size_t k = b + i;
      const T z = T(0);
      ((T*)st.steer)[k] = z; ((T*)st.acc)[k] = z; ((T*)st.impact_x)[k] = z; ((T*)st.impact_y)[k] = z;
      st.crashed[k] = 0; st.has_impact[k] = 0;
      if (i == 0) {
        st.kind[k] = TTRL_MDP; st.lane_change[k] = 0;
        X[k] = T(ex); Y[k] = T(ey); Hh[k] = T(eh); Vv[k] = T(cfg.ego_speed);
        const int ln = closest_lane_index<CV>(R, ex, ey, eh);
        st.lane[k] = st.target_lane[k] = ln;
        const int si = speed_to_index(P, cfg.ego_speed);
        st.speed_index[k] = si;
        TS[k] = T(P.target_speeds[si]);
        TM[k] = z; DL[k] = T(4);
      } else if (i < nv) {
        st.kind[k] = TTRL_IDM; st.lane_change[k] = (uint8_t)cfg.lane_change;
        X[k] = T(px); Y[k] = T(py); Hh[k] = T(ph); Vv[k] = T(sp); TS[k] = T(sp);
        const int ln = closest_lane_index<CV>(R, px, py, ph);
        st.lane[k] = st.target_lane[k] = ln;
        st.speed_index[k] = -1;
        TM[k] = T(pymod((px + py) * 3.141592653589793, P.lane_change_delay));
        DL[k] = T(delta);
      } else {
        st.kind[k] = TTRL_ABSENT; st.lane_change[k] = 0;
        X[k] = Y[k] = Hh[k] = Vv[k] = TS[k] = TM[k] = z;
        DL[k] = T(4); st.lane[k] = st.target_lane[k] = 0; st.speed_index[k] = -1;
      }
    }
  }
#ifdef TTRL_RESET_TRACE
  RT();
  if (lane == 0 && (env % 512) == 7)
    printf("reset env %d: seed %lld draws %lld place %lld store %lld (wall clocks, 100 MHz)\n", env, tr[1] - tr[0],
           tr[2] - tr[1], tr[3] - tr[2], tr[4] - tr[3]);
#endif
#undef RT
  if (__any(reject)) {  // a rejected integers() draw shifts the stream: replay this env in order
    __threadfence_block();
    __syncthreads();
    if (lane == 0) {
      Pcg g;
      g.st = s0; g.inc = inc; g.has32 = false; g.u32 = 0;
      reset_env_serial<T>(st, R, P, cfg, g, env);
    }
  }
}

// IntersectionEnv._agent_reward / _is_terminated / _is_truncated (intersection_env.py:78-119) for one
// env's ego (has_ego false: no controlled vehicle) and AbstractEnv.step's time += 1 / policy
// frequency (abstract.py:239); ego_speed / ego_crashed: the info's speed / crashed (abstract.py:169-186),
// of slot 0 when there is no ego.  rewards_kernel and simulate_kernel (ttrl_env_step) both call it.
template <typename T>
__device__ __forceinline__ void step_tail(const ttrl_lane_table_t& R, const LaneT<T>* L, const ttrl_reward_cfg_t& cfg,
                                          int env, bool has_ego, T x, T y, T v, int l, bool crashed, T v0,
                                          bool crashed0, double* __restrict__ time, double time_inc,
                                          float* __restrict__ reward, uint8_t* __restrict__ term,
                                          uint8_t* __restrict__ trunc, float* __restrict__ comp,
                                          T* __restrict__ ego_speed, uint8_t* __restrict__ ego_crashed) {
  double t = time[env];
  if (time_inc != 0.0) {
    t += time_inc;
    time[env] = t;
  }
  if (ego_speed) {
    ego_speed[env] = has_ego ? v : v0;
    ego_crashed[env] = has_ego ? crashed : crashed0;
  }
  trunc[env] = (uint8_t)(t >= cfg.duration);
  if (!has_ego) {
    reward[env] = 0.f; term[env] = 0;
    if (comp) for (int q = 0; q < 4; ++q) comp[(size_t)env * 4 + q] = 0.f;
    return;
  }
  const T hs = clip(lmap(v, T(cfg.speed_lo), T(cfg.speed_hi), T(0), T(1)), T(0), T(1));
  T s, r;
  lane_local(*L, x, y, s, r);  // L: the ego's lane l
  const bool onroad = fabs(r) <= T(R.width[l]) / T(2) + T(0) && -T(5) <= s && s < T(R.length[l]) + T(5);
  const bool arrived = R.exit_lane[l] && s >= T(cfg.exit_distance);
  T rw = T(cfg.collision_reward) * T(crashed ? 1 : 0) + T(cfg.high_speed_reward) * hs +
         T(cfg.arrived_reward) * T(arrived ? 1 : 0);
  if (arrived) rw = T(cfg.arrived_reward);
  rw *= T(onroad ? 1 : 0);
  if (cfg.normalize_reward) rw = lmap(rw, T(cfg.collision_reward), T(cfg.arrived_reward), T(0), T(1));
  reward[env] = (float)rw;
  term[env] = (uint8_t)(crashed || arrived || (cfg.offroad_terminal && !onroad));
  if (comp) {
    float* c = comp + (size_t)env * 4;
    c[0] = crashed ? 1.f : 0.f; c[1] = (float)hs; c[2] = arrived ? 1.f : 0.f; c[3] = onroad ? 1.f : 0.f;
  }
}

template <typename T>
__global__ void rewards_kernel(ttrl_state_t st, ttrl_lane_table_t R, ttrl_reward_cfg_t cfg, double* __restrict__ time,
                               double time_inc, float* __restrict__ reward, uint8_t* __restrict__ term,
                               uint8_t* __restrict__ trunc, float* __restrict__ comp, T* __restrict__ ego_speed,
                               uint8_t* __restrict__ ego_crashed) {
  const int env = blockIdx.x * blockDim.x + threadIdx.x;
  if (env >= st.n_envs) return;
  const size_t b = (size_t)env * st.n_veh;
  int ego = 0;
  while (ego < st.n_veh && st.kind[b + ego] != TTRL_MDP) ++ego;
  const bool has_ego = ego < st.n_veh;
  const size_t k = b + (has_ego ? ego : 0);
  const int l = st.lane[k];
  LaneT<T> L{};
  if (has_ego) L = make_lane<T>(R, l);
  step_tail<T>(R, &L, cfg, env, has_ego, ((const T*)st.x)[k], ((const T*)st.y)[k],
               ((const T*)st.speed)[k], l, st.crashed[k] != 0, ((const T*)st.speed)[b], st.crashed[b] != 0, time,
               time_inc, reward, term, trunc, comp, ego_speed, ego_crashed);
}

// ------------------------------------------------------------ the intersection scenario
// IntersectionEnv (intersection_env.py:131-362) scene management: one wavefront per env, the
// env's slots on the lanes (chunks of 64 when n_veh > 64).  The vehicle list is sequential by
// nature (spawns append, clears keep list order, every draw advances the env's np_random), so
// every lane replays the same numpy Generator in lockstep -- identical state, identical draws,
// identical (uniform) rejection loops -- while the per-slot work is spread over the lanes:
// clearing and compacting the rows (coalesced), the spawn's distance test (ballot), the
// closest-lane search (one road lane per SIMD lane, first-minimum argmin by xor-shuffles).

// Every field of one vehicle row, for compaction in registers.
template <typename T> struct Row {
  T f[11];  // x, y, heading, speed, target_speed, timer, delta, steer, acc, impact_x, impact_y
  int32_t lane, tgt, sidx, route_road, route_lane;  // the 4 int8 route entries packed in one word each
  uint8_t kind, crashed, has_impact, lane_change, yielding;
  int8_t route_n;
};
template <typename T>
__device__ __forceinline__ T* real_field(const ttrl_state_t& st, int q) {
  void* const p[11] = {st.x, st.y, st.heading, st.speed, st.target_speed, st.timer, st.delta,
                       st.steer, st.acc, st.impact_x, st.impact_y};
  return (T*)p[q];
}
template <typename T>
__device__ __forceinline__ Row<T> row_load(const ttrl_state_t& st, size_t k) {
  Row<T> r;
#pragma unroll
  for (int q = 0; q < 11; ++q) r.f[q] = real_field<T>(st, q)[k];
  r.lane = st.lane[k]; r.tgt = st.target_lane[k]; r.sidx = st.speed_index[k];
  r.route_road = ((const int32_t*)st.route_road)[k];  // TTRL_ROUTE_MAX == 4 int8 entries
  r.route_lane = ((const int32_t*)st.route_lane)[k];
  r.kind = st.kind[k]; r.crashed = st.crashed[k]; r.has_impact = st.has_impact[k];
  r.lane_change = st.lane_change[k]; r.yielding = st.yielding[k]; r.route_n = st.route_n[k];
  return r;
}
template <typename T>
__device__ __forceinline__ void row_store(const ttrl_state_t& st, size_t k, const Row<T>& r) {
#pragma unroll
  for (int q = 0; q < 11; ++q) real_field<T>(st, q)[k] = r.f[q];
  st.lane[k] = r.lane; st.target_lane[k] = r.tgt; st.speed_index[k] = r.sidx;
  ((int32_t*)st.route_road)[k] = r.route_road;
  ((int32_t*)st.route_lane)[k] = r.route_lane;
  st.kind[k] = r.kind; st.crashed[k] = r.crashed; st.has_impact[k] = r.has_impact;
  st.lane_change[k] = r.lane_change; st.yielding[k] = r.yielding; st.route_n[k] = r.route_n;
}
template <typename T>
__device__ __forceinline__ Row<T> row_absent() {  // an empty slot, as BatchState initialises it
  Row<T> r;
#pragma unroll
  for (int q = 0; q < 11; ++q) r.f[q] = T(0);
  r.f[6] = T(4);  // IDMVehicle.DELTA
  r.lane = r.tgt = 0; r.sidx = -1; r.route_road = r.route_lane = -1;
  r.kind = TTRL_ABSENT; r.crashed = r.has_impact = r.lane_change = r.yielding = 0; r.route_n = -1;
  return r;
}
// Survivors (present slots whose keep bit is set) move down in list order; the tail is cleared.
// keep: bit j of word j / 64.  All of a chunk's rows are read before any is written; writes
// only go to slots <= the one read, so earlier chunks are never read again.
template <typename T>
__device__ void wave_compact(const ttrl_state_t& st, size_t base, const unsigned long long* keep, int lane) {
  int w = 0;
  for (int c0 = 0; c0 < st.n_veh; c0 += 64) {
    const int j = c0 + lane;
    const bool in = j < st.n_veh;
    Row<T> r;
    bool live = false;
    if (in) {
      r = row_load<T>(st, base + j);
      live = r.kind != TTRL_ABSENT && ((keep[c0 >> 6] >> lane) & 1ull);
    }
    const unsigned long long m = __ballot(live);
    const int dst = w + __popcll(m & ((1ull << lane) - 1ull));
    __syncthreads();
    if (live) row_store<T>(st, base + dst, r);
    w += __popcll(m);
  }
  __syncthreads();
  for (int j = w + lane; j < st.n_veh; j += 64) row_store<T>(st, base + j, row_absent<T>());
  __syncthreads();
}
__device__ __forceinline__ int wave_count(const ttrl_state_t& st, size_t base, int lane) {
  int n = 0;
  for (int c0 = 0; c0 < st.n_veh; c0 += 64)
    n += __popcll(__ballot(c0 + lane < st.n_veh && st.kind[base + c0 + lane] != TTRL_ABSENT));
  return n;
}
// RoadNetwork.get_closest_lane_index road.py:55-71 (distance_with_heading lane.py:132-147, first
// minimum), one network lane per SIMD lane; the result is uniform.
__device__ int wave_closest_lane(const ttrl_lane_table_t& R, double x, double y, double h, int lane) {
  double best = K<double>::inf();
  int bl = 0x7fffffff;
  for (int l0 = 0; l0 < R.n_lanes; l0 += 64) {
    const int l = l0 + lane;
    if (l < R.n_lanes) {
      const LaneT<double> L = make_lane<double>(R, l);
      double s, r;
      lane_local(L, x, y, s, r);
      const double ang = fabs(wrap_to_pi(h - heading_at(L, s)));
      double a = s - R.length[l]; if (!(a > 0)) a = 0;
      double c = 0 - s; if (!(c > 0)) c = 0;
      const double d = fabs(r) + a + c + 1.0 * ang;
      if (d < best || (d == best && l < bl)) { best = d; bl = l; }
    }
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const double od = __shfl_xor(best, off);
    const int ol = __shfl_xor(bl, off);
    if (od < best || (od == best && ol < bl)) { best = od; bl = ol; }
  }
  return bl == 0x7fffffff ? 0 : bl;
}
// ControlledVehicle.plan_route_to controller.py:71-87 (shortest_path precomputed on the host):
// the packed route words of a vehicle on `lane` heading for corner `corner`.
__device__ __forceinline__ void plan_route(const ttrl_lane_table_t& R, const ttrl_ix_cfg_t& C, int lane, int corner,
                                           int32_t& rr, int32_t& rl, int8_t& rn) {
  const int road = R.road[lane], node = R.road_to[road];
  const int n = C.path_len[node][corner] > 0 ? C.path_len[node][corner] : 0;
  int8_t a[TTRL_ROUTE_MAX], b[TTRL_ROUTE_MAX];
  for (int q = 0; q < TTRL_ROUTE_MAX; ++q) a[q] = b[q] = -1;
  a[0] = (int8_t)road; b[0] = (int8_t)R.lane_id[lane];
  for (int q = 0; q < n; ++q) a[1 + q] = C.path_road[node][corner][q];
  rr = rl = 0;
  for (int q = 0; q < TTRL_ROUTE_MAX; ++q) {
    rr |= (int32_t)(uint8_t)a[q] << (8 * q);
    rl |= (int32_t)(uint8_t)b[q] << (8 * q);
  }
  rn = (int8_t)(1 + n);
}
// IntersectionEnv._spawn_vehicle intersection_env.py:320-348 (IDMVehicle.make_on_lane
// objects.py:68-89, IDMVehicle.__init__ behavior.py:48-64, randomize_behavior :66-69).
// Uniform across the wave: every lane holds the same generator and makes the same draws.
template <typename T, typename PP>
__device__ void wave_spawn(const ttrl_state_t& st, const ttrl_lane_table_t& R, const PP& P,
                           const ttrl_ix_cfg_t& C, Pcg& g, size_t base, int lane, double longitudinal, double pos_dev,
                           double speed_dev, double prob, bool go_straight) {
  if (pcg_double(g) > prob) return;
  int route[2];
  pcg_choice_noreplace(g, 4, 2, route);
  if (go_straight) route[1] = (route[0] + 2) % 4;
  const int l = C.entry_lane[route[0]];
  const double lon = longitudinal + C.spawn_offset + pcg_normal(g) * pos_dev;
  const double sp = C.spawn_speed + pcg_normal(g) * speed_dev;
  const LaneT<double> L = make_lane<double>(R, l);
  double px, py;
  lane_position(L, lon, 0.0, px, py);
  const double ph = heading_at(L, lon);
  bool near = false;
  for (int j = lane; j < st.n_veh; j += 64) {
    const size_t k = base + j;
    if (st.kind[k] == TTRL_ABSENT) continue;
    const double dx = (double)((const T*)st.x)[k] - px, dy = (double)((const T*)st.y)[k] - py;
    near |= sqrt(dx * dx + dy * dy) < C.spawn_clear_distance;
  }
  if (__any(near)) return;
  const int n = wave_count(st, base, lane);
  const double delta = C.delta_lo + (C.delta_hi - C.delta_lo) * pcg_double(g);  // drawn even with no slot left
  if (n >= st.n_veh) return;
  const int cl = wave_closest_lane(R, px, py, ph, lane);
  if (lane == 0) {
    Row<T> r = row_absent<T>();
    r.kind = TTRL_IDM; r.lane_change = 1;
    r.f[0] = T(px); r.f[1] = T(py); r.f[2] = T(ph); r.f[3] = T(sp); r.f[4] = T(sp);
    r.f[5] = T(pymod((px + py) * 3.141592653589793, P.lane_change_delay));
    r.f[6] = T(delta);
    r.lane = r.tgt = cl;
    plan_route(R, C, cl, route[1], r.route_road, r.route_lane, r.route_n);
    row_store<T>(st, base + n, r);
  }
  __syncthreads();
}

// IntersectionEnv._reset, part 1: np_random = default_rng(SeedSequence(entropy)), _make_road's
// fresh RegulatedRoad (steps 0, no vehicles), the n-1 initial spawns (intersection_env.py:262-263).
template <typename T>
__global__ void __launch_bounds__(64) ix_begin_kernel(ttrl_state_t st, ttrl_lane_table_t R, ttrl_params_t P,
                                                      ttrl_ix_cfg_t C, const unsigned* __restrict__ words,
                                                      int n_words, const uint8_t* __restrict__ mask) {
  const int env = blockIdx.x, lane = threadIdx.x;
  if (mask && !mask[env]) return;
  const size_t base = (size_t)env * st.n_veh;
  unsigned long long s4[4];
  SeedSeq::pcg64_seed(words + (size_t)env * n_words, n_words, s4);
  Pcg g;
  g.st = U128{s4[0], s4[1]}; g.inc = U128{s4[2], s4[3]}; g.has32 = false; g.u32 = 0;
  for (int j = lane; j < st.n_veh; j += 64) row_store<T>(st, base + j, row_absent<T>());
  if (lane == 0) st.reg_steps[env] = 0;
  __syncthreads();
  for (int t = 0; t < C.initial_vehicle_count - 1; ++t)
    wave_spawn<T>(st, R, P, C, g, base, lane, C.init_longitudinal[t], 1.0, 1.0, C.spawn_probability, false);
  if (lane == 0) rng_store(g, st.rng + (size_t)env * TTRL_RNG_WORDS);
}

// IntersectionEnv._reset, part 2 (after the warm-up frames): the challenger, the ego
// MDPVehicle appended after the traffic, and the removal of the vehicles within 20 m of it,
// which skips the vehicle after each removed one (list.remove while iterating, :308-312).
template <typename T>
__global__ void __launch_bounds__(64) ix_finish_kernel(ttrl_state_t st, ttrl_lane_table_t R, ttrl_params_t P,
                                                       ttrl_ix_cfg_t C, const uint8_t* __restrict__ mask) {
  const int env = blockIdx.x, lane = threadIdx.x;
  if (mask && !mask[env]) return;
  const size_t base = (size_t)env * st.n_veh;
  uint64_t* w = st.rng + (size_t)env * TTRL_RNG_WORDS;
  Pcg g = rng_load(w);
  wave_spawn<T>(st, R, P, C, g, base, lane, C.challenger_longitudinal, C.challenger_position_deviation,
                C.challenger_speed_deviation, 1.0, true);
  const int dest = C.ego_destination >= 0 ? C.ego_destination : 1 + (int)pcg_bounded(g, 3);
  const double lon = C.ego_longitudinal + C.ego_deviation * (1.0 + pcg_normal(g));
  int n = wave_count(st, base, lane);
  if (n >= st.n_veh) n = st.n_veh - 1;  // no slot left: the last vehicle gives way to the ego
  const LaneT<double> L = make_lane<double>(R, C.ego_lane);
  double ex, ey;
  lane_position(L, lon, 0.0, ex, ey);
  const double eh = heading_at(L, C.ego_heading_s);
  const int cl = wave_closest_lane(R, ex, ey, eh, lane);
  if (lane == 0) {
    Row<T> r = row_absent<T>();
    r.kind = TTRL_MDP;
    r.f[0] = T(ex); r.f[1] = T(ey); r.f[2] = T(eh); r.f[3] = T(C.ego_speed);
    r.lane = r.tgt = cl;
    r.sidx = speed_to_index(P, C.ego_speed);
    r.f[4] = T(P.target_speeds[r.sidx]);
    plan_route(R, C, cl, dest, r.route_road, r.route_lane, r.route_n);
    row_store<T>(st, base + n, r);
  }
  __syncthreads();
  // which vehicles are within ego_clear_distance (the ego's stored position, as the reference's
  // np.linalg.norm(v.position - ego_vehicle.position))
  const T exs = ((const T*)st.x)[base + n], eys = ((const T*)st.y)[base + n];
  unsigned long long nearw[4] = {0, 0, 0, 0};
  for (int c0 = 0; c0 < n + 1; c0 += 64) {
    const int j = c0 + lane;
    bool nr = false;
    if (j < n) {
      const double dx = (double)((const T*)st.x)[base + j] - (double)exs;
      const double dy = (double)((const T*)st.y)[base + j] - (double)eys;
      nr = sqrt(dx * dx + dy * dy) < C.ego_clear_distance;
    }
    nearw[c0 >> 6] = __ballot(nr);
  }
  // list.remove while iterating (uniform on every lane): positions shift left after a removal
  // while the iterator index still advances, so the vehicle after each removed one is skipped
  unsigned long long keep[4] = {~0ull, ~0ull, ~0ull, ~0ull};
  {
    int i = 0, removed = 0;  // i: iterator index; list position p holds slot p + removed (until then)
    int j = 0;               // the slot at position i
    while (true) {
      j = i + removed;
      if (j > n) break;
      if (j != n && ((nearw[j >> 6] >> (j & 63)) & 1ull)) {
        keep[j >> 6] &= ~(1ull << (j & 63));
        ++removed;
      }
      ++i;
    }
  }
  wave_compact<T>(st, base, keep, lane);
  if (lane == 0) rng_store(g, w);
}

// IntersectionEnv.step tail (intersection_env.py:135-139): _clear_vehicles (:350-362) keeps the
// controlled vehicle and every vehicle neither leaving (an "il"->"o" lane within 4 lengths of its
// end) nor without a route, in list order; then _spawn_vehicle(spawn_probability).
template <typename T, typename PP>
__device__ void ix_clear_spawn_env(const ttrl_state_t& st, const ttrl_lane_table_t& R, const PP& P,
                                   const ttrl_ix_cfg_t& C, int env, int lane) {
  const size_t base = (size_t)env * st.n_veh;
  unsigned long long keep[4] = {~0ull, ~0ull, ~0ull, ~0ull};
  for (int c0 = 0; c0 < st.n_veh; c0 += 64) {
    const int j = c0 + lane;
    bool drop = false;
    if (j < st.n_veh && st.kind[base + j] == TTRL_IDM) {
      const size_t k = base + j;
      const int l = st.lane[k];
      T s, r;
      lane_local(make_lane<T>(R, l), ((const T*)st.x)[k], ((const T*)st.y)[k], s, r);
      const bool leaving = R.exit_lane[l] && s >= T(R.length[l]) - T(C.leave_margin);
      drop = leaving || st.route_n[k] < 0;
    }
    keep[c0 >> 6] = ~__ballot(drop);
  }
  wave_compact<T>(st, base, keep, lane);
  uint64_t* w = st.rng + (size_t)env * TTRL_RNG_WORDS;
  Pcg g = rng_load(w);
  wave_spawn<T>(st, R, P, C, g, base, lane, 0.0, 1.0, 1.0, C.spawn_probability, false);
  if (lane == 0) rng_store(g, w);
}

// Position of the n-th (0-based) set bit of m (n < popcount(m)).
__device__ __forceinline__ int nth_set_bit(unsigned long long m, int n) {
  int pos = 0;
#pragma unroll
  for (int w = 32; w >= 1; w >>= 1) {
    const int c = __popcll(m & ((1ull << w) - 1ull));
    if (n >= c) { n -= c; m >>= w; pos += w; }
  }
  return pos;
}

// wave_closest_lane over the NS-lane segment of one env (NS <= 64, a power of two; the result is
// uniform on the segment): the same float64 distances and first-minimum rule.
template <int NS>
__device__ int seg_closest_lane(const ttrl_lane_table_t& R, double x, double y, double h, int i) {
  double best = K<double>::inf();
  int bl = 0x7fffffff;
  for (int l = i; l < R.n_lanes; l += NS) {
    const LaneT<double> L = make_lane<double>(R, l);
    double s, r;
    lane_local(L, x, y, s, r);
    const double ang = fabs(wrap_to_pi(h - heading_at(L, s)));
    double a = s - R.length[l]; if (!(a > 0)) a = 0;
    double c = 0 - s; if (!(c > 0)) c = 0;
    const double d = fabs(r) + a + c + 1.0 * ang;
    if (d < best || (d == best && l < bl)) { best = d; bl = l; }
  }
#pragma unroll
  for (int off = NS / 2; off >= 1; off >>= 1) {
    const double od = __shfl_xor(best, off);
    const int ol = __shfl_xor(bl, off);
    if (od < best || (od == best && ol < bl)) { best = od; bl = ol; }
  }
  return bl == 0x7fffffff ? 0 : bl;
}

// The simulate launch's epilogue under ttrl_ix_env_step (one wavefront per workgroup, an env's
// vehicles on NS lanes of it), from the final LDS state -- IntersectionEnv.step after the frames
// (intersection_env.py:135-139 over abstract.py:224-250) and the auto-reset (abstract.py:188-214):
//  (a) the step tail (step_tail: time, reward, terminated, truncated, info terms), as ttrl_env_step;
//  (b) the Kinematics observation of the final state (kin_observe, np_random's shuffle) into so.obs
//      and, for an env that goes on, into ie.obs2 as well (its next observation);
//  (c) an env that goes on: _clear_vehicles (:350-362) -- the IDM vehicles on an exit lane within
//      leave_margin of its end or without a route are dropped, the others keep list order (each
//      lane takes the row of the i-th kept slot by lane shuffles) -- then (d) _spawn_vehicle
//      (:320-348), every lane of the env replaying its np_random (wave_spawn's draws; the 15 m test
//      by a segment ballot, the closest lane by segment shuffles);
//  (e) the rows to HBM: an env that goes on every field of every slot (absent ones as row_absent,
//      as wave_compact leaves them); a finished env takes its spare scene instead, row par[e] * E + e
//      (every field, the regulation and np_random words included; its final rows are discarded, as
//      the reset discards them), and (f) the tail's counters (episode words, parity, time, masks);
//  (g) a finished env's first observation of the new scene into ie.obs2 (kin_observe from HBM);
//  (h) the live counts (live, live_env).
// Bit for bit ttrl_env_step followed by ttrl_ix_step_tail (test_fused_tail_equals_the_separate_tail,
// test_overlapped_resets_equal_in_place_resets).
template <typename T, int NS, int EPW>
__device__ __forceinline__ void ix_epilogue(const View<T>& V, const ttrl_state_t& st, const ttrl_lane_table_t& R,
                                            const ParamsT<T>& P, const StepOut& so, const IxEpi& ie, int le, int i,
                                            int env, bool env_on, bool slot, size_t k, int me, int eb, int reg,
                                            T& timer, T& steer, T& acc, T& ix, T& iy, int& sidx) {
  static_assert(NS * EPW == 64, "the fused tail runs on the one-wavefront road-network instance");
  constexpr unsigned long long SEG = NS == 64 ? ~0ull : ((1ull << NS) - 1);
  constexpr int M = EPW * NS;
  const int N = st.n_veh, E = st.n_envs;
  const int kind = V.kind[me];
  const bool present = kind != TTRL_ABSENT;
  char* scr = (char*)V.afree;
  T* s_key = (T*)scr;
  int(*s_perm)[64] = (int(*)[64])(scr + ((sizeof(T) * M + 15) & ~(size_t)15));
  int(*s_p)[64] = s_perm + EPW;
  int* s_cnt = (int*)(s_p + EPW);
  int* s_ego = s_cnt + EPW;
  if (i == 0 && env_on) st.reg_steps[env] = reg;
  // (a) the step tail; V.nitem[le] (dead since the last act phase): -1 the env goes on, else the
  // spare slot a finished env takes (-2: no env)
  if (i == 0) s_ego[le] = N;
  __syncthreads();
  if (present && kind == TTRL_MDP) atomicMin(&s_ego[le], i);
  __syncthreads();
  if (i == 0) {
    int st8 = -2;
    if (env_on) {
      const int ego = s_ego[le];
      step_tail<T>(R, V.lanes + (ego < N ? (int)V.lane[eb + ego] : 0), so.rcfg, env, ego < N, V.x[eb + ego % N],
                   V.y[eb + ego % N], V.v[eb + ego % N], (int)V.lane[eb + ego % N],
                   (V.flags[eb + ego % N] & FL_CRASHED) != 0, V.v[eb], (V.flags[eb] & FL_CRASHED) != 0, so.time,
                   so.time_inc, so.reward, so.term, so.trunc, so.comp, (T*)so.ego_speed, so.ego_crashed);
      st8 = !so.term[env] && !so.trunc[env] ? -1 : (int)ie.par[env];
    }
    V.nitem[le] = st8;
  }
  __syncthreads();
  const int pslot = V.nitem[le];
  const bool go_on = pslot == -1, fin = pslot >= 0;
  // (b) the observation of the final state
  {
    auto ego_of = [&](int ego, T& ex, T& ey, T& eh, T& ev, T& ec, T& es, int& elane) {
      ex = V.x[eb + ego]; ey = V.y[eb + ego]; eh = V.h[eb + ego]; ev = V.v[eb + ego]; elane = V.lane[eb + ego];
      ec = V.ch[eb + ego]; es = V.sh[eb + ego];
    };
    kin_observe<T, NS, EPW>(st, V.lanes, P, so.kcfg, env_on, env, V.x[me], V.y[me], V.h[me], V.v[me], V.ch[me],
                            V.sh[me], (int)V.lane[me], present, present && kind == TTRL_MDP, ego_of, s_key, s_cnt,
                            s_ego, s_perm, s_p, so.obs, so.ids, go_on ? ie.obs2 : nullptr,
                            go_on ? ie.ids2 : nullptr);
  }
  __syncthreads();  // the shuffle's np_random words (lane 0 of the env) before the spawn reads them
  // (c) _clear_vehicles: the kept slots of an env that goes on
  bool keep = present;
  if (go_on && present && kind == TTRL_IDM) {
    const int l = V.lane[me];
    T s, r;
    lane_local(V.lanes[l], V.x[me], V.y[me], s, r);
    const bool leaving = R.exit_lane[l] && s >= T(R.length[l]) - T(ie.C.leave_margin);
    keep = !(leaving || V.rn[me] < 0);
  }
  const unsigned long long kb = (__ballot(keep) >> eb) & SEG;
  const int cnt = __popcll(kb);
  // lane i takes the row of the i-th kept slot (i >= cnt: absent); the other envs keep their rows
  const int src = go_on ? (i < cnt ? nth_set_bit(kb, i) : -1) : i;
  const int sl = eb + (src < 0 ? i : src);
  {
    const T nx = __shfl(V.x[me], sl), ny = __shfl(V.y[me], sl), nv = __shfl(V.v[me], sl);
    const T nts = __shfl(V.ts[me], sl), nh = __shfl(V.h[me], sl), nd = __shfl(V.delta[me], sl);
    const int nb = __shfl((int)((unsigned)V.kind[me] | (unsigned)V.flags[me] << 8 | (unsigned)(uint8_t)V.lane[me] << 16 |
                                (unsigned)(uint8_t)V.tgt[me] << 24), sl);
    const int nrr = __shfl(((const int32_t*)V.rroad)[me], sl), nrl = __shfl(((const int32_t*)V.rlane)[me], sl);
    const int nrn = __shfl((int)V.rn[me], sl);
    const T nti = __shfl(timer, sl), nst = __shfl(steer, sl), nac = __shfl(acc, sl);
    const T nix = __shfl(ix, sl), niy = __shfl(iy, sl);
    const int nsi = __shfl(sidx, sl);
    if (go_on) {
      if (src >= 0) {
        V.x[me] = nx; V.y[me] = ny; V.v[me] = nv; V.ts[me] = nts; V.h[me] = nh; V.delta[me] = nd;
        V.kind[me] = (uint8_t)(nb & 0xff); V.flags[me] = (uint8_t)((nb >> 8) & 0xff);
        V.lane[me] = (int8_t)((nb >> 16) & 0xff); V.tgt[me] = (int8_t)((nb >> 24) & 0xff);
        ((int32_t*)V.rroad)[me] = nrr; ((int32_t*)V.rlane)[me] = nrl; V.rn[me] = (int8_t)nrn;
        timer = nti; steer = nst; acc = nac; ix = nix; iy = niy; sidx = nsi;
      } else {
        V.kind[me] = TTRL_ABSENT;
      }
    }
  }
  __syncthreads();
  // (d) _spawn_vehicle (wave_spawn's draws, in order), every lane of an env that goes on alike
  int n_live = cnt;
  if (go_on) {
    uint64_t* w = st.rng + (size_t)env * TTRL_RNG_WORDS;
    Pcg g = rng_load(w);
    if (!(pcg_double(g) > ie.C.spawn_probability)) {
      int route[2];
      pcg_choice_noreplace(g, 4, 2, route);
      const int l = ie.C.entry_lane[route[0]];
      const double lon = 0.0 + ie.C.spawn_offset + pcg_normal_body(g) * 1.0;
      const double sp = ie.C.spawn_speed + pcg_normal_body(g) * 1.0;
      const LaneT<double> L = make_lane<double>(R, l);
      double px, py;
      lane_position(L, lon, 0.0, px, py);
      const double ph = heading_at(L, lon);
      bool near = false;
      if (i < cnt) {
        const double dx = (double)V.x[me] - px, dy = (double)V.y[me] - py;
        near = sqrt(dx * dx + dy * dy) < ie.C.spawn_clear_distance;
      }
      if (((__ballot(near) >> eb) & SEG) == 0) {
        const double delta = ie.C.delta_lo + (ie.C.delta_hi - ie.C.delta_lo) * pcg_double(g);  // drawn even with no slot left
        if (cnt < N) {
          const int cl = seg_closest_lane<NS>(R, px, py, ph, i);
          if (i == cnt) {
            int32_t rr, rl;
            int8_t rn;
            plan_route(R, ie.C, cl, route[1], rr, rl, rn);
            V.x[me] = T(px); V.y[me] = T(py); V.h[me] = T(ph); V.v[me] = T(sp); V.ts[me] = T(sp);
            V.delta[me] = T(delta);
            V.kind[me] = TTRL_IDM; V.flags[me] = FL_LC;
            V.lane[me] = (int8_t)cl; V.tgt[me] = (int8_t)cl;
            ((int32_t*)V.rroad)[me] = rr; ((int32_t*)V.rlane)[me] = rl; V.rn[me] = rn;
            timer = T(pymod((px + py) * 3.141592653589793, ie.lane_change_delay));
            steer = acc = ix = iy = T(0);
            sidx = -1;
          }
          n_live = cnt + 1;
        }
      }
    }
    if (i == 0) rng_store(g, w);
  }
  // (e) the rows to HBM
  if (slot && go_on) {  // every field of every slot (compaction moved them)
    const int kd = V.kind[me];
    const int fl = V.flags[me];
    Row<T> r = row_absent<T>();
    if (kd != TTRL_ABSENT) {
      r.f[0] = V.x[me]; r.f[1] = V.y[me]; r.f[2] = V.h[me]; r.f[3] = V.v[me]; r.f[4] = V.ts[me];
      r.f[5] = timer; r.f[6] = V.delta[me]; r.f[7] = steer; r.f[8] = acc; r.f[9] = ix; r.f[10] = iy;
      r.lane = V.lane[me]; r.tgt = V.tgt[me]; r.sidx = sidx;
      r.route_road = ((const int32_t*)V.rroad)[me]; r.route_lane = ((const int32_t*)V.rlane)[me];
      r.kind = (uint8_t)kd; r.crashed = (fl & FL_CRASHED) ? 1 : 0; r.has_impact = (fl & FL_IMPACT) ? 1 : 0;
      r.lane_change = (fl & FL_LC) ? 1 : 0; r.yielding = (fl & FL_YIELD) ? 1 : 0; r.route_n = V.rn[me];
    }
    row_store<T>(st, k, r);
  }
  if (fin) {  // the spare scene: every slot of row par * E + env (copy_env_rows' fields)
    const int row = pslot * E + env;
    Row<T> r = row_absent<T>();
    if (i < N) {
      r = row_load<T>(ie.spare, (size_t)row * N + i);
      row_store<T>(st, k, r);
    }
    if (i == 0) st.reg_steps[env] = ie.spare.reg_steps[row];
    if (i < TTRL_RNG_WORDS) st.rng[(size_t)env * TTRL_RNG_WORDS + i] = ie.spare.rng[(size_t)row * TTRL_RNG_WORDS + i];
    // the new scene into the env's (dead) view rows for its observation: the same values (g) would
    // load back from HBM
    V.x[me] = r.f[0]; V.y[me] = r.f[1]; V.h[me] = r.f[2]; V.v[me] = r.f[3];
    V.lane[me] = (int8_t)(i < N ? r.lane : 0);
    V.kind[me] = (uint8_t)(i < N ? r.kind : TTRL_ABSENT);
    const SinCos<T> sc = k_sincos(r.f[2]);
    V.ch[me] = sc.c; V.sh[me] = sc.s;
  }
  // (f) the tail's counters (ix_step_tail_kernel's)
  if (i == 0 && env_on) {
    ie.done[env] = fin ? 1 : 0;
    for (int q = 0; q < ie.K; ++q) ie.spare_mask[(size_t)q * E + env] = fin && q == pslot;
    if (fin) {
      const int row = pslot * E + env;
      ie.ent[(size_t)env * ie.nw + ie.nw - 1] += 1u;
      ie.spare_ent[(size_t)row * ie.nw + ie.nw - 1] += (unsigned)ie.K;  // this slot's next episode
      ie.par[env] = (uint8_t)(pslot + 1 == ie.K ? 0 : pslot + 1);
      so.time[env] = 0.0;
    }
  }
  __syncthreads();  // the new scenes' view rows and np_random words
  // (g) a finished env's first observation of its new scene (ix_step_tail_kernel's, from the view)
  {
    const int kd = V.kind[me];
    const bool pr = fin && kd != TTRL_ABSENT;
    if (fin) n_live = __popcll((__ballot(pr) >> eb) & SEG);
    auto ego_of = [&](int ego, T& ex, T& ey, T& eh, T& ev, T& ec, T& es, int& elane) {
      ex = V.x[eb + ego]; ey = V.y[eb + ego]; eh = V.h[eb + ego]; ev = V.v[eb + ego]; elane = V.lane[eb + ego];
      ec = V.ch[eb + ego]; es = V.sh[eb + ego];
    };
    kin_observe<T, NS, EPW>(st, V.lanes, P, so.kcfg, fin, env, V.x[me], V.y[me], V.h[me], V.v[me], V.ch[me], V.sh[me],
                            (int)V.lane[me], pr, pr && kd == TTRL_MDP, ego_of, s_key, s_cnt, s_ego, s_perm, s_p,
                            ie.obs2, ie.ids2);
  }
  // (h) the live counts
  if (env_on && i == 0) {
    if (ie.live_env) ie.live_env[env] = n_live;
    if (ie.live) atomicAdd(ie.live, (unsigned long long)n_live);
  }
}

template <typename T>
__global__ void __launch_bounds__(64) ix_clear_spawn_kernel(ttrl_state_t st, ttrl_lane_table_t R, ttrl_params_t P,
                                                            ttrl_ix_cfg_t C, const uint8_t* __restrict__ mask) {
  const int env = blockIdx.x, lane = threadIdx.x;
  if (mask && !mask[env]) return;
  ix_clear_spawn_env<T>(st, R, P, C, env, lane);
}

// One row of every field (per-env route / regulation / rng words included) from src row ks to dst
// row kd, the slots on the lanes of one wavefront.
template <typename T>
__device__ __forceinline__ void copy_env_rows(const ttrl_state_t& dst, const ttrl_state_t& src, int env_dst,
                                              int env_src, int lane) {
  const size_t bd = (size_t)env_dst * dst.n_veh, bs = (size_t)env_src * src.n_veh;
  const bool net = dst.route_road && src.route_road;
  for (int j = lane; j < dst.n_veh; j += 64) {
    const size_t kd = bd + j, ks = bs + j;
#pragma unroll
    for (int q = 0; q < 11; ++q) real_field<T>(dst, q)[kd] = real_field<T>(src, q)[ks];
    dst.lane[kd] = src.lane[ks]; dst.target_lane[kd] = src.target_lane[ks]; dst.speed_index[kd] = src.speed_index[ks];
    dst.kind[kd] = src.kind[ks]; dst.crashed[kd] = src.crashed[ks]; dst.has_impact[kd] = src.has_impact[ks];
    dst.lane_change[kd] = src.lane_change[ks];
    if (net) {
      ((int32_t*)dst.route_road)[kd] = ((const int32_t*)src.route_road)[ks];
      ((int32_t*)dst.route_lane)[kd] = ((const int32_t*)src.route_lane)[ks];
      dst.route_n[kd] = src.route_n[ks];
      dst.yielding[kd] = src.yielding[ks];
    }
  }
  if (lane == 0 && dst.reg_steps && src.reg_steps) dst.reg_steps[env_dst] = src.reg_steps[env_src];
  if (lane < TTRL_RNG_WORDS && dst.rng && src.rng)
    dst.rng[(size_t)env_dst * TTRL_RNG_WORDS + lane] = src.rng[(size_t)env_src * TTRL_RNG_WORDS + lane];
}

// VecIntersectionEnv.step after the fused simulate / observation / reward launch, with auto-reset
// from scenes reset ahead of time (the spare rows), in one launch, one wavefront per env:
// - an env that goes on runs IntersectionEnv.step's tail (_clear_vehicles, _spawn_vehicle;
//   intersection_env.py:135-139) and keeps its observation row (obs_in -> obs_out);
// - a finished env (terminated | truncated) is reset (AbstractEnv.reset, abstract.py:188-214): it
//   takes the spare scene of its parity slot (prepared from default_rng([seed words, episode]) by
//   ttrl_ix_reset), so its clear / spawn -- which the reset discards with the rest of the finished
//   scene, rows and np_random alike -- is skipped; its episode counter advances, the consumed spare
//   row's counter advances by two (that row's next scene is two episodes on) and is flagged in
//   spare_mask for the side stream's reset, the parity flips, time is zeroed, and the first
//   observation of the new scene is written to obs_out / ids_out (kin_observe, one slot per lane).
struct IxTail {
  ttrl_state_t spare;  // K * E rows: slot p of env e is row p * E + e
  int K;               // spare slots per env, taken in rotation
  const uint8_t* term;
  const uint8_t* trunc;
  uint8_t* par;        // [E] the next slot each env takes
  uint32_t* ent;       // [E][nw] entropy words, the episode counter last
  uint32_t* spare_ent; // [K * E][nw]
  int nw;
  double* time;
  uint8_t* done;       // [E] out
  uint8_t* spare_mask; // [2E] out
  ttrl_kin_cfg_t kcfg;
  bool obs;
  const float* obs_in;
  float* obs_out;
  const int32_t* ids_in;
  int32_t* ids_out;
  unsigned long long* live;  // optional: += the vehicles present after the tail (the next step's)
  int32_t* live_env;         // optional [E]: each env's vehicles present after the tail
};

// The env's present vehicles after the tail: added to *t.live (one atomic per env) and / or
// written to t.live_env[env] (the next step's dispatch order, ix_order_kernel).
template <typename T>
__device__ __forceinline__ void ix_count_live(const ttrl_state_t& st, const IxTail& t, int env, int lane) {
  __syncthreads();  // the tail's writes to kind (clear / spawn, or the copied rows) are the block's own
  const int N = st.n_veh;
  int c = 0;
  for (int q0 = 0; q0 < N; q0 += 64)
    c += __popcll(__ballot(q0 + lane < N && st.kind[(size_t)env * N + q0 + lane] != TTRL_ABSENT));
  if (lane == 0) {
    if (t.live) atomicAdd(t.live, (unsigned long long)c);
    if (t.live_env) t.live_env[env] = c;
  }
}

// Counting sort of the P groups of G consecutive envs by key_of(p) in [0, NB) ascending (ties in
// any order), into order[0, P * G): one workgroup.  h: NB ints of LDS.
constexpr int ORDER_BUCKETS = 320;  // 5 per lane of the scanning wave
template <typename KeyFn>
__device__ void sort_groups(int32_t* __restrict__ order, int P, int G, int* h, KeyFn key_of) {
  const int tid = threadIdx.x;
  for (int b = tid; b < ORDER_BUCKETS; b += blockDim.x) h[b] = 0;
  __syncthreads();
  for (int p = tid; p < P; p += blockDim.x) atomicAdd(&h[key_of(p)], 1);
  __syncthreads();
  if (tid < 64) {  // exclusive prefix over the buckets
    int v[5], sum = 0;
    for (int j = 0; j < 5; ++j) { v[j] = h[tid * 5 + j]; sum += v[j]; }
    int inc = sum;
    for (int d = 1; d < 64; d <<= 1) {
      const int o = __shfl_up(inc, d);
      if (tid >= d) inc += o;
    }
    int run = inc - sum;
    for (int j = 0; j < 5; ++j) { h[tid * 5 + j] = run; run += v[j]; }
  }
  __syncthreads();
  for (int p = tid; p < P; p += blockDim.x) {
    const int pos = atomicAdd(&h[key_of(p)], 1);
    for (int q = 0; q < G; ++q) order[pos * G + q] = p * G + q;
  }
}

// The next step's dispatch order (one workgroup, after the tail): the simulate launch's groups of G
// consecutive envs (its workgroups), heaviest first by the group's live vehicles (kmax <= 256).
// The hardware dispatches workgroups in slot order, so the long-running groups start first and the
// cheap ones fill in behind them -- and behind the warm-up waves of the spare resets a step launch
// finds resident (the slots they hold push the last-dispatched groups into a second round).  The
// step's results do not depend on the order (test_dispatch_order_leaves_results_unchanged,
// test_overlapped_resets_equal_in_place_resets).  order: [0, E) out, [E, 2E) the tail's live counts.
__global__ void __launch_bounds__(1024) ix_order_kernel(int32_t* __restrict__ order, int E, int G, int kmax) {
  __shared__ int h[ORDER_BUCKETS];
  const int32_t* live = order + E;
  sort_groups(order, E / G, G, h, [&](int p) {
    int k = 0;
    for (int q = 0; q < G; ++q) k += live[p * G + q];
    return kmax - min(max(k, 0), kmax);  // descending
  });
}

template <typename T>
__global__ void __launch_bounds__(64) ix_step_tail_kernel(ttrl_state_t st, ttrl_lane_table_t R, ttrl_params_t P,
                                                          ttrl_ix_cfg_t C, IxTail t) {
  __shared__ T s_key[64];
  __shared__ int s_cnt[1], s_ego[1];
  __shared__ int s_perm[1][64], s_p[1][64];
  __shared__ LaneT<T> s_lanes[LMAX];
  const int env = blockIdx.x, lane = threadIdx.x;
  const int E = st.n_envs, N = st.n_veh;
  const bool d = t.term[env] || t.trunc[env];
  const int V = t.kcfg.vehicles_count, F = t.kcfg.n_features;
  if (!d) {
    if (lane == 0) {
      t.done[env] = 0;
      for (int q = 0; q < t.K; ++q) t.spare_mask[q * E + env] = 0;
    }
    if (t.obs) {  // the row observed by the fused launch stays this step's observation
      for (int q = lane; q < V * F; q += 64) t.obs_out[(size_t)env * V * F + q] = t.obs_in[(size_t)env * V * F + q];
      if (t.ids_out)
        for (int q = lane, W = V > 1 ? V - 1 : 1; q < W; q += 64) t.ids_out[(size_t)env * W + q] = t.ids_in[(size_t)env * W + q];
    }
    ix_clear_spawn_env<T>(st, R, P, C, env, lane);
    if (t.live || t.live_env) ix_count_live<T>(st, t, env, lane);
    return;
  }
  const int p = t.par[env];
  const int row = p * E + env;
  copy_env_rows<T>(st, t.spare, env, row, lane);
  if (lane == 0) {
    t.done[env] = 1;
    t.ent[(size_t)env * t.nw + t.nw - 1] += 1u;
    t.spare_ent[(size_t)row * t.nw + t.nw - 1] += (unsigned)t.K;  // this slot's next episode
    for (int q = 0; q < t.K; ++q) t.spare_mask[q * E + env] = q == p;
    t.par[env] = (uint8_t)(p + 1 == t.K ? 0 : p + 1);
    t.time[env] = 0.0;
  }
  if (t.live || t.live_env) ix_count_live<T>(st, t, env, lane);
  if (!t.obs) return;
  if (lane < R.n_lanes) s_lanes[lane] = make_lane<T>(R, lane);
  __syncthreads();  // the copied rows (and rng words) are the block's own writes: visible after the barrier
  const size_t k = (size_t)env * N + lane;
  T x = T(0), y = T(0), h = T(0), v = T(0);
  int ln = 0;
  bool present = false, mdp = false;
  if (lane < N) {
    x = ((const T*)st.x)[k]; y = ((const T*)st.y)[k]; h = ((const T*)st.heading)[k];
    v = ((const T*)st.speed)[k]; ln = st.lane[k];
    present = st.kind[k] != TTRL_ABSENT;
    mdp = st.kind[k] == TTRL_MDP;
  }
  auto ego_of = [&](int ego, T& ex, T& ey, T& eh, T& ev, T& ec, T& es, int& elane) {
    const size_t k0 = (size_t)env * N + ego;
    ex = ((const T*)st.x)[k0]; ey = ((const T*)st.y)[k0]; eh = ((const T*)st.heading)[k0];
    ev = ((const T*)st.speed)[k0]; elane = st.lane[k0];
    const SinCos<T> sc = k_sincos(eh);
    ec = sc.c; es = sc.s;
  };
  const SinCos<T> sc = k_sincos(h);
  kin_observe<T, 64, 1>(st, s_lanes, P, t.kcfg, true, env, x, y, h, v, sc.c, sc.s, ln, present, mdp, ego_of, s_key,
                        s_cnt, s_ego, s_perm, s_p, t.obs_out, t.ids_out);
}

// Masked whole-env copy (double-buffered resets): one workgroup per env, the slots on the lanes.
template <typename T>
__global__ void __launch_bounds__(64) copy_envs_kernel(ttrl_state_t dst, ttrl_state_t src,
                                                       const uint8_t* __restrict__ mask) {
  const int env = blockIdx.x, lane = threadIdx.x;
  if (!mask[env]) return;
  copy_env_rows<T>(dst, src, env, env, lane);
}

// ------------------------------------------------------------------- launch helpers
// A network beyond one road, or a RegulatedRoad: the simulate kernel's NET_GRAPH instance.
bool is_graph(const ttrl_lane_table_t& R) { return R.n_roads > 1 || R.regulation_frequency > 0; }

// TTRL_OK, a negative TTRL_E_* code, or EMPTY (> 0: no env, nothing to do -- the entry points
// then return TTRL_OK before looking at buffers an empty batch need not have)
#ifndef TTRL_KERNEL_ONLY  // host launchers
constexpr int EMPTY = 1;
int check_state(const ttrl_state_t* s, const ttrl_lane_table_t* R) {
  if (!s || !R) return TTRL_E_ARG;
  if (s->dtype != TTRL_F32 && s->dtype != TTRL_F64) return TTRL_E_ARG;
  if (s->n_envs < 0 || s->n_veh < 1 || s->n_veh > 256) return TTRL_E_ARG;
  if (s->n_envs == 0) return EMPTY;
  if (R->n_lanes < 1 || R->n_lanes > LMAX) return TTRL_E_ARG;
  if (R->n_roads < 1 || R->n_roads > TTRL_MAX_ROADS || R->regulation_frequency < 0) return TTRL_E_ARG;
  for (int l = 0; l < R->n_lanes; ++l)  // topology consistent (lanes of a road contiguous, in id order)
    if (R->road[l] < 0 || R->road[l] >= R->n_roads || R->road_first[R->road[l]] + R->lane_id[l] != l ||
        R->lane_id[l] >= R->road_n[R->road[l]])
      return TTRL_E_ARG;
  if (is_graph(*R) && (!s->route_road || !s->route_lane || !s->route_n || !s->yielding || !s->reg_steps))
    return TTRL_E_ARG;
  const void* ptrs[] = {s->x, s->y, s->heading, s->speed, s->target_speed, s->timer, s->delta, s->steer, s->acc,
                        s->impact_x, s->impact_y, s->lane, s->target_lane, s->speed_index, s->kind, s->crashed,
                        s->has_impact, s->lane_change};
  for (const void* p : ptrs)
    if (!p) return TTRL_E_ARG;
  return TTRL_OK;
}

int slots_for(int n) { return n <= 32 ? 32 : n <= 64 ? 64 : n <= 128 ? 128 : 256; }

// The reset instance for a road: CV = false when every lane is straight along +x (the highway).
template <typename T>
void launch_reset(const ttrl_state_t& s, const ttrl_lane_table_t& R, const ttrl_params_t& P,
                  const ttrl_reset_cfg_t& cfg, const unsigned long long* pcg, unsigned* words, int n_words,
                  const uint8_t* mask, const AutoReset& ar, hipStream_t st) {
  bool curved = false;
  for (int l = 0; l < R.n_lanes; ++l)
    curved |= R.type[l] != TTRL_LANE_STRAIGHT || R.dir_x[l] != 1.0 || R.dir_y[l] != 0.0;
  if (curved)
    hipLaunchKernelGGL((reset_wave_kernel<T, true>), dim3(s.n_envs), dim3(64), 0, st, s, R, P, cfg, pcg, words,
                       n_words, mask, ar);
  else
    hipLaunchKernelGGL((reset_wave_kernel<T, false>), dim3(s.n_envs), dim3(64), 0, st, s, R, P, cfg, pcg, words,
                       n_words, mask, ar);
}

int launch_status() { return hipGetLastError() == hipSuccess ? TTRL_OK : TTRL_E_LAUNCH; }

// ttrl_env_step's tail scratch (the observation's keys, rows and counts; simulate_body's epilogue)
// fits the act phase's block it overlays (dead after the last frame).
template <typename T>
bool tail_fits(const ViewLayout& o, int EPW, int NS) {
  const size_t M = (size_t)EPW * NS;
  const size_t need = ((sizeof(T) * M + 15) & ~(size_t)15) + 2 * sizeof(int) * 64 * EPW + 2 * sizeof(int) * EPW;
  return o.afree + need <= o.item + sizeof(short) * 2 * M;
}

// SIMDs (4 per CU on CDNA) of the device the launch stream belongs to (the null stream: the
// current device), cached per device id; the cache is atomic, so host threads driving different
// devices may launch concurrently.
int simds_of_stream_device(hipStream_t stream) {
  static std::atomic<int> cache[16];
  int dev = -1;
  if (stream) {
    hipDevice_t d = -1;
    if (hipStreamGetDevice(stream, &d) == hipSuccess) dev = d;
  }
  if (dev < 0 && (hipGetDevice(&dev) != hipSuccess || dev < 0)) return 1024;
  if (dev < 16) {
    const int c = cache[dev].load(std::memory_order_relaxed);
    if (c) return c;
  }
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
  if (dev < 16) cache[dev].store(4 * cus, std::memory_order_relaxed);
  return 4 * cus;
}

template <typename T, int NS, int EPW>
int launch_sim(const ttrl_state_t& s, const ttrl_lane_table_t& R, const ttrl_params_t& P, const int32_t* actions,
               const uint8_t* mask, int frames, double dt, int mode, int ablate, hipStream_t stream,
               const StepOut& ob) {
  const int blocks = (s.n_envs + EPW - 1) / EPW;
  if (blocks == 0) return TTRL_OK;
  const bool graph = is_graph(R);
  // the NET_STRAIGHT instance: at most STRAIGHT_LANE_CAP straight lanes along +x; any other road
  // (curved, rotated or wider) runs the NET_CURVED instance, which handles every lane class
  bool curved = R.n_lanes > STRAIGHT_LANE_CAP;
  for (int l = 0; l < R.n_lanes; ++l)
    curved |= R.type[l] != TTRL_LANE_STRAIGHT || R.dir_x[l] != 1.0 || R.dir_y[l] != 0.0;
  const size_t lds = host_view_bytes(sizeof(T) == 8 ? TTRL_F64 : TTRL_F32, EPW, NS,
                                     graph || curved ? R.n_lanes : STRAIGHT_LANE_CAP, graph,
                                     !graph && !curved && sorted_view(NS, EPW, NET_STRAIGHT));
  if (ob.obs || ob.reward) {  // the tail's scratch must fit the dead block it overlays (it does for every NS)
    const ViewLayout o = view_layout<T>(EPW, NS, graph || curved ? R.n_lanes : STRAIGHT_LANE_CAP, graph,
                                        !graph && !curved && sorted_view(NS, EPW, NET_STRAIGHT));
    if (!tail_fits<T>(o, EPW, NS)) return TTRL_E_UNSUPPORTED;
  }
  const ParamsT<T> PT = params_for<T>(P);
  if constexpr (NS == 32 && EPW == 2) {
    // every wave resident at 2 per SIMD: the 2-wave register budget (no spills) costs no occupancy
    if (!graph && !curved && blocks <= 2 * simds_of_stream_device(stream)) {
      hipLaunchKernelGGL((simulate_kernel<T, NS, EPW, NET_STRAIGHT, 2>), dim3(blocks), dim3(NS * EPW), lds, stream,
                         s, R, PT, actions, mask, frames, dt, mode, ablate, ob);
      return launch_status();
    }
  }
  if (graph)
    hipLaunchKernelGGL((simulate_kernel<T, NS, EPW, NET_GRAPH>), dim3(blocks), dim3(NS * EPW), lds, stream, s, R, PT,
                       actions, mask, frames, dt, mode, ablate, ob);
  else if (curved)
    hipLaunchKernelGGL((simulate_kernel<T, NS, EPW, NET_CURVED>), dim3(blocks), dim3(NS * EPW), lds, stream, s, R,
                       PT, actions, mask, frames, dt, mode, ablate, ob);
  else
    hipLaunchKernelGGL((simulate_kernel<T, NS, EPW, NET_STRAIGHT>), dim3(blocks), dim3(NS * EPW), lds, stream, s, R,
                       PT, actions, mask, frames, dt, mode, ablate, ob);
  return launch_status();
}

template <typename T>
int dispatch_sim(const ttrl_state_t& s, const ttrl_lane_table_t& R, const ttrl_params_t& P, const int32_t* actions,
                 const uint8_t* mask, int frames, double dt, int mode, int ablate, hipStream_t stream,
                 const StepOut& ob) {
  switch (slots_for(s.n_veh)) {
    case 32: return launch_sim<T, 32, 2>(s, R, P, actions, mask, frames, dt, mode, ablate, stream, ob);
    case 64: return launch_sim<T, 64, 1>(s, R, P, actions, mask, frames, dt, mode, ablate, stream, ob);
    case 128: return launch_sim<T, 128, 1>(s, R, P, actions, mask, frames, dt, mode, ablate, stream, ob);
    default: return launch_sim<T, 256, 1>(s, R, P, actions, mask, frames, dt, mode, ablate, stream, ob);
  }
}

// ttrl_ix_env_step's launch: the one-wavefront road-network instance with the fused tail (IxEpi)
template <typename T, int NS, int EPW>
int launch_sim_ix(const ttrl_state_t& s, const ttrl_lane_table_t& R, const ttrl_params_t& P, const int32_t* actions,
                  int frames, double dt, hipStream_t stream, const StepOut& ob, const IxEpi& ie) {
  const int blocks = (s.n_envs + EPW - 1) / EPW;
  if (blocks == 0) return TTRL_OK;
  const ViewLayout o = view_layout<T>(EPW, NS, R.n_lanes, true, false);
  if (!tail_fits<T>(o, EPW, NS)) return TTRL_E_UNSUPPORTED;
  hipLaunchKernelGGL((simulate_ix_kernel<T, NS, EPW>), dim3(blocks), dim3(NS * EPW), o.total, stream, s, R,
                     params_for<T>(P), actions, frames, dt, ob, ie);
  return launch_status();
}

// ttrl_env_step_grid's launch: the straight one-env instance (sorted view) with the OccupancyGrid
// epilogue, its scratch over the view's blocks dead after the last frame (the own-state and the
// frame-transient blocks: 8.8 KB per float64 128-slot env for the 8 KB a 7 x 32 x 32 grid and its
// cfg need; the block grows if a grid needs more)
template <typename T, int NS>
int launch_sim_grid(const ttrl_state_t& s, const ttrl_lane_table_t& R, const ttrl_params_t& P, const int32_t* actions,
                    int frames, double dt, hipStream_t stream, const StepOut& ob, GridEpi ge) {
  if (s.n_envs == 0) return TTRL_OK;
  const ViewLayout o = view_layout<T>(1, NS, STRAIGHT_LANE_CAP, false, true);
  if (!tail_fits<T>(o, 1, NS)) return TTRL_E_UNSUPPORTED;
  ge.scr = (uint32_t)o.own;
  const size_t need =
      o.own + ((sizeof(ttrl_grid_cfg_t) + 15) & ~(size_t)15) + grid_scratch_bytes(ge.cfg, s.n_veh, sizeof(T));
  const size_t lds = need > o.total ? (need + 15) & ~(size_t)15 : o.total;
  if (lds > 64 * 1024) return TTRL_E_UNSUPPORTED;
  hipLaunchKernelGGL((simulate_grid_kernel<T, NS>), dim3(s.n_envs), dim3(NS), lds, stream, s, R, params_for<T>(P),
                     actions, frames, dt, ob, ge);
  return launch_status();
}

// The road and slot count run the straight one-env-per-workgroup instance with a sorted view
// (launch_sim's choice for 64 and 128 slots on <= STRAIGHT_LANE_CAP straight lanes along +x).
bool grid_fusable(const ttrl_state_t& s, const ttrl_lane_table_t& R) {
  if (is_graph(R) || R.n_lanes > STRAIGHT_LANE_CAP) return false;
  for (int l = 0; l < R.n_lanes; ++l)
    if (R.type[l] != TTRL_LANE_STRAIGHT || R.dir_x[l] != 1.0 || R.dir_y[l] != 0.0) return false;
  const int ns = slots_for(s.n_veh);
  return ns == 64 || ns == 128;
}

int run_sim(const ttrl_state_t* s, const ttrl_lane_table_t* R, const ttrl_params_t* P, const int32_t* actions,
            int frames, double dt, int mode, void* stream, int ablate = 0, const uint8_t* mask = nullptr,
            const StepOut* ob = nullptr) {
  int rc = check_state(s, R);
  if (rc) return rc < 0 ? rc : TTRL_OK;
  if (!P || frames < 0 || P->n_target_speeds < 1 || P->n_target_speeds > 8) return TTRL_E_ARG;
  hipStream_t st = (hipStream_t)stream;
  const StepOut none{};
  const StepOut& o = ob ? *ob : none;
  return s->dtype == TTRL_F64 ? dispatch_sim<double>(*s, *R, *P, actions, mask, frames, dt, mode, ablate, st, o)
                              : dispatch_sim<float>(*s, *R, *P, actions, mask, frames, dt, mode, ablate, st, o);
}

int check_grid_cfg(const ttrl_grid_cfg_t* cfg, const float* out) {
  if (!cfg || !out || cfg->n_features < 1 || cfg->n_features > TTRL_N_FEATURES || cfg->shape_x < 1 ||
      cfg->shape_y < 1 || cfg->step_x <= 0 || cfg->step_y <= 0)
    return TTRL_E_ARG;
  for (int c = 0; c < cfg->n_features; ++c)
    if (cfg->features[c] < 0 || cfg->features[c] >= TTRL_N_FEATURES) return TTRL_E_ARG;
  return TTRL_OK;
}

int check_kin_cfg(const ttrl_state_t* s, const ttrl_kin_cfg_t* cfg) {
  if (!cfg || cfg->vehicles_count < 1 || cfg->n_features < 1 || cfg->n_features > TTRL_N_FEATURES) return TTRL_E_ARG;
  if (cfg->order_shuffled < 0 || cfg->order_shuffled > 2) return TTRL_E_ARG;
  if (cfg->order_shuffled == 2 && (!s->rng || cfg->vehicles_count - 1 > 64)) return TTRL_E_ARG;
  for (int c = 0; c < cfg->n_features; ++c)
    if (cfg->features[c] < 0 || cfg->features[c] >= TTRL_F_ON_ROAD) return TTRL_E_ARG;
  return TTRL_OK;
}

template <typename T, int NS, int EPW>
int launch_nbr(const ttrl_state_t& s, const ttrl_lane_table_t& R, const ttrl_params_t& P, const int32_t* q,
               int32_t* f, int32_t* r, hipStream_t stream) {
  const int blocks = (s.n_envs + EPW - 1) / EPW;
  if (blocks == 0) return TTRL_OK;
  const size_t lds = host_view_bytes(sizeof(T) == 8 ? TTRL_F64 : TTRL_F32, EPW, NS, R.n_lanes);
  hipLaunchKernelGGL((neighbours_kernel<T, NS, EPW>), dim3(blocks), dim3(NS * EPW), lds, stream, s, R, P, q, f, r);
  return launch_status();
}

template <typename T>
int dispatch_nbr(const ttrl_state_t& s, const ttrl_lane_table_t& R, const ttrl_params_t& P, const int32_t* q,
                 int32_t* f, int32_t* r, hipStream_t st) {
  switch (slots_for(s.n_veh)) {
    case 32: return launch_nbr<T, 32, 2>(s, R, P, q, f, r, st);
    case 64: return launch_nbr<T, 64, 1>(s, R, P, q, f, r, st);
    case 128: return launch_nbr<T, 128, 1>(s, R, P, q, f, r, st);
    default: return launch_nbr<T, 256, 1>(s, R, P, q, f, r, st);
  }
}

template <typename T, int NS, int EPW>
int launch_kin(const ttrl_state_t& s, const ttrl_lane_table_t& R, const ttrl_params_t& P, const ttrl_kin_cfg_t& c,
               const uint8_t* mask, float* out, int32_t* ids, hipStream_t stream) {
  const int blocks = (s.n_envs + EPW - 1) / EPW;
  if (blocks == 0) return TTRL_OK;
  hipLaunchKernelGGL((kinematics_obs_kernel<T, NS, EPW>), dim3(blocks), dim3(NS * EPW), 0, stream, s, R, P, c, mask,
                     out, ids);
  return launch_status();
}

template <typename T>
int dispatch_kin(const ttrl_state_t& s, const ttrl_lane_table_t& R, const ttrl_params_t& P, const ttrl_kin_cfg_t& c,
                 const uint8_t* mask, float* out, int32_t* ids, hipStream_t st) {
  switch (slots_for(s.n_veh)) {
    case 32: return launch_kin<T, 32, 2>(s, R, P, c, mask, out, ids, st);
    case 64: return launch_kin<T, 64, 1>(s, R, P, c, mask, out, ids, st);
    case 128: return launch_kin<T, 128, 1>(s, R, P, c, mask, out, ids, st);
    default: return launch_kin<T, 256, 1>(s, R, P, c, mask, out, ids, st);
  }
}

#endif  // TTRL_KERNEL_ONLY
#ifdef TTRL_KERNEL_ONLY  // kernel-development builds (tools/asmstat.py): the highway instances only
void* const kernel_only_refs[] = {(void*)&simulate_kernel<double, 64, 1, NET_STRAIGHT>,
                                  (void*)&simulate_kernel<float, 64, 1, NET_STRAIGHT>};
#endif
}  // namespace

#ifndef TTRL_KERNEL_ONLY

// ===================================================================== C ABI
extern "C" {

int ttrl_abi_version(void) { return TTRL_ABI_VERSION; }

int ttrl_meta_action(const ttrl_state_t* s, const ttrl_lane_table_t* road, const ttrl_params_t* p,
                     const int32_t* actions, void* stream) {
  if (!actions) return TTRL_E_ARG;
  return run_sim(s, road, p, actions, 1, 0.0, MODE_META, stream);
}

int ttrl_road_act(const ttrl_state_t* s, const ttrl_lane_table_t* road, const ttrl_params_t* p, void* stream) {
  return run_sim(s, road, p, nullptr, 1, 0.0, MODE_ACT, stream);
}

int ttrl_road_step(const ttrl_state_t* s, const ttrl_lane_table_t* road, const ttrl_params_t* p, double dt,
                   void* stream) {
  return run_sim(s, road, p, nullptr, 1, dt, MODE_STEP, stream);
}

int ttrl_simulate(const ttrl_state_t* s, const ttrl_lane_table_t* road, const ttrl_params_t* p,
                  const int32_t* actions, int32_t frames, double dt, void* stream) {
  return run_sim(s, road, p, actions, frames, dt, MODE_META | MODE_ACT | MODE_STEP, stream);
}

int ttrl_env_step_grid(const ttrl_state_t* s, const ttrl_lane_table_t* road, const ttrl_params_t* p,
                       const int32_t* actions, int32_t frames, double dt, const ttrl_grid_cfg_t* grid_cfg, float* grid,
                       const ttrl_reward_cfg_t* reward_cfg, double* time, double time_inc, float* reward,
                       uint8_t* terminated, uint8_t* truncated, float* components, void* ego_speed,
                       uint8_t* ego_crashed, const int32_t* action_lut, int32_t n_action_lut, void* stream) {
  int rc = check_state(s, road);
  if (rc) return rc < 0 ? rc : TTRL_OK;
  if (check_grid_cfg(grid_cfg, grid)) return TTRL_E_ARG;
  if (!grid_fusable(*s, *road)) {  // two launches: the step, then grid_obs_kernel
    rc = ttrl_env_step(s, road, p, actions, frames, dt, nullptr, nullptr, nullptr, reward_cfg, time, time_inc, reward,
                       terminated, truncated, components, ego_speed, ego_crashed, nullptr, action_lut, n_action_lut,
                       stream);
    return rc ? rc : ttrl_observe_grid(s, road, p, grid_cfg, grid, stream);
  }
  if (!p || frames < 0 || p->n_target_speeds < 1 || p->n_target_speeds > 8) return TTRL_E_ARG;
  if (reward_cfg && (!time || !reward || !terminated || !truncated || (!ego_speed) != (!ego_crashed)))
    return TTRL_E_ARG;
  if (n_action_lut < 0 || n_action_lut > 8 || (n_action_lut > 0 && !action_lut)) return TTRL_E_ARG;
  StepOut so{};
  for (int q = 0; q < n_action_lut; ++q) {
    if (action_lut[q] < TTRL_LANE_LEFT || action_lut[q] > TTRL_SLOWER) return TTRL_E_ARG;
    so.lut[q] = (int8_t)action_lut[q];
  }
  so.n_lut = n_action_lut;
  if (reward_cfg) {
    so.rcfg = *reward_cfg; so.time = time; so.time_inc = time_inc; so.reward = reward; so.term = terminated;
    so.trunc = truncated; so.comp = components; so.ego_speed = ego_speed; so.ego_crashed = ego_crashed;
  }
  GridEpi ge{};
  ge.cfg = *grid_cfg;
  ge.out = grid;
  hipStream_t st = (hipStream_t)stream;
  const bool wide = slots_for(s->n_veh) == 128;
  if (s->dtype == TTRL_F64)
    return wide ? launch_sim_grid<double, 128>(*s, *road, *p, actions, frames, dt, st, so, ge)
                : launch_sim_grid<double, 64>(*s, *road, *p, actions, frames, dt, st, so, ge);
  return wide ? launch_sim_grid<float, 128>(*s, *road, *p, actions, frames, dt, st, so, ge)
              : launch_sim_grid<float, 64>(*s, *road, *p, actions, frames, dt, st, so, ge);
}

int ttrl_env_step(const ttrl_state_t* s, const ttrl_lane_table_t* road, const ttrl_params_t* p, const int32_t* actions,
                  int32_t frames, double dt, const ttrl_kin_cfg_t* obs_cfg, float* obs, int32_t* obs_ids,
                  const ttrl_reward_cfg_t* reward_cfg, double* time, double time_inc, float* reward,
                  uint8_t* terminated, uint8_t* truncated, float* components, void* ego_speed, uint8_t* ego_crashed,
                  const int32_t* order, const int32_t* action_lut, int32_t n_action_lut, void* stream) {
  int rc = check_state(s, road);
  if (rc) return rc < 0 ? rc : TTRL_OK;
  if ((!obs_cfg) != (!obs) || (obs_cfg && check_kin_cfg(s, obs_cfg))) return TTRL_E_ARG;
  if (reward_cfg && (!time || !reward || !terminated || !truncated || (!ego_speed) != (!ego_crashed)))
    return TTRL_E_ARG;
  if (n_action_lut < 0 || n_action_lut > 8 || (n_action_lut > 0 && !action_lut)) return TTRL_E_ARG;
  StepOut so{};
  for (int q = 0; q < n_action_lut; ++q) {
    if (action_lut[q] < TTRL_LANE_LEFT || action_lut[q] > TTRL_SLOWER) return TTRL_E_ARG;
    so.lut[q] = (int8_t)action_lut[q];
  }
  so.n_lut = n_action_lut;
  if (obs_cfg) { so.kcfg = *obs_cfg; so.obs = obs; so.ids = obs_ids; }
  if (reward_cfg) {
    so.rcfg = *reward_cfg; so.time = time; so.time_inc = time_inc; so.reward = reward; so.term = terminated;
    so.trunc = truncated; so.comp = components; so.ego_speed = ego_speed; so.ego_crashed = ego_crashed;
  }
  so.order = order;
  return run_sim(s, road, p, actions, frames, dt, MODE_META | MODE_ACT | MODE_STEP, stream, 0, nullptr, &so);
}

/* Diagnostic only (not in include/): the simulate kernel's LDS view bytes per workgroup. */
long ttrl_diag_view_bytes(int32_t dtype, int32_t epw, int32_t ns, int32_t n_lanes, int32_t graph, int32_t sorted) {
  return (long)host_view_bytes(dtype, epw, ns, n_lanes, graph != 0, sorted != 0);
}

/* Diagnostic only (not in include/): the flattened enforcement's queue capacity of a road-network
 * view (0: the serial pair loop runs). */
long ttrl_diag_rq_cap(int32_t dtype, int32_t epw, int32_t ns, int32_t n_lanes) {
  return (long)(dtype == TTRL_F64 ? view_layout<double>(epw, ns, n_lanes, true, false).rq_cap
                                  : view_layout<float>(epw, ns, n_lanes, true, false).rq_cap);
}

/* Diagnostic only (not in include/): the fused loop with phases ablated, for profiling. */
int ttrl_diag_simulate(const ttrl_state_t* s, const ttrl_lane_table_t* road, const ttrl_params_t* p,
                       const int32_t* actions, int32_t frames, double dt, int32_t ablate, void* stream) {
#ifndef TTRL_DIAG_ABLATE
  if (ablate != 0) return TTRL_E_UNSUPPORTED;  // a -DTTRL_DIAG_ABLATE build of the library ablates phases
#endif
  return run_sim(s, road, p, actions, frames, dt, MODE_META | MODE_ACT | MODE_STEP, stream, ablate);
}

#if defined(TTRL_PHASE_TIMING) || defined(TTRL_WAVE_TRACE)
// Diagnostic build only: read and clear the per-phase cycle sums (PH_SLOTS u64: 20 phases,
// project_items' 5 steps, the regulation's 5 steps and 2 event counts).
int ttrl_diag_phase_read(unsigned long long* out) {
  unsigned long long z[PH_SLOTS] = {};
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_phase), sizeof(z)) != hipSuccess) return TTRL_E_LAUNCH;
  return hipMemcpyToSymbol(HIP_SYMBOL(g_phase), z, sizeof(z)) == hipSuccess ? TTRL_OK : TTRL_E_LAUNCH;
}
// ... each wave's phase cycles of the last launch (PHASE_TIMING builds): n x 30 u32
int ttrl_diag_wave_phases(unsigned* out, int n) {
  if (n > WTRACE_MAX) n = WTRACE_MAX;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wphase), sizeof(unsigned) * PH_SLOTS * n) == hipSuccess ? TTRL_OK
                                                                                                  : TTRL_E_LAUNCH;
}
// ... and the per-wave trace of the last launch: n x (start, end, hw_id | xcc_id << 32)
int ttrl_diag_wave_read(unsigned long long* out, int n) {
  if (n > WTRACE_MAX) n = WTRACE_MAX;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wtrace), sizeof(unsigned long long) * 3 * n) == hipSuccess
             ? TTRL_OK : TTRL_E_LAUNCH;
}
#endif

int ttrl_neighbours(const ttrl_state_t* s, const ttrl_lane_table_t* road, const int32_t* query_lane,
                    int32_t* front, int32_t* rear, void* stream) {
  int rc = check_state(s, road);
  if (rc) return rc < 0 ? rc : TTRL_OK;
  if (!front || !rear) return TTRL_E_ARG;
  ttrl_params_t P{};
  P.lane_vehicle_length = 5.0;  // AbstractLane.VEHICLE_LENGTH
  hipStream_t st = (hipStream_t)stream;
  return s->dtype == TTRL_F64 ? dispatch_nbr<double>(*s, *road, P, query_lane, front, rear, st)
                              : dispatch_nbr<float>(*s, *road, P, query_lane, front, rear, st);
}

int ttrl_observe_kinematics_masked(const ttrl_state_t* s, const ttrl_lane_table_t* road, const ttrl_params_t* p,
                                   const ttrl_kin_cfg_t* cfg, const uint8_t* mask, float* out, int32_t* ids,
                                   void* stream) {
  int rc = check_state(s, road);
  if (rc) return rc < 0 ? rc : TTRL_OK;
  if (!p || !out || check_kin_cfg(s, cfg)) return TTRL_E_ARG;
  hipStream_t st = (hipStream_t)stream;
  return s->dtype == TTRL_F64 ? dispatch_kin<double>(*s, *road, *p, *cfg, mask, out, ids, st)
                              : dispatch_kin<float>(*s, *road, *p, *cfg, mask, out, ids, st);
}

int ttrl_observe_kinematics(const ttrl_state_t* s, const ttrl_lane_table_t* road, const ttrl_params_t* p,
                            const ttrl_kin_cfg_t* cfg, float* out, int32_t* ids, void* stream) {
  return ttrl_observe_kinematics_masked(s, road, p, cfg, nullptr, out, ids, stream);
}

int ttrl_observe_grid(const ttrl_state_t* s, const ttrl_lane_table_t* road, const ttrl_params_t* p,
                      const ttrl_grid_cfg_t* cfg, float* out, void* stream) {
  int rc = check_state(s, road);
  if (rc) return rc < 0 ? rc : TTRL_OK;
  if (!p || check_grid_cfg(cfg, out)) return TTRL_E_ARG;
  const size_t lds = grid_scratch_bytes(*cfg, s->n_veh, s->dtype == TTRL_F64 ? 8 : 4);
  if (lds > 160 * 1024) return TTRL_E_UNSUPPORTED;
  if (s->n_envs == 0) return TTRL_OK;
  hipStream_t st = (hipStream_t)stream;
  // one thread per slot (64 .. 256): smaller blocks for fewer vehicles keep more envs in flight
  // (4096 x 128: 2 waves per env, all 4096 envs resident at once)
  const int nt = s->n_veh <= 64 ? 64 : (s->n_veh <= 128 ? 128 : (s->n_veh <= 192 ? 192 : 256));
  if (s->dtype == TTRL_F64)
    hipLaunchKernelGGL(grid_obs_kernel<double>, dim3(s->n_envs), dim3(nt), lds, st, *s, *road, *p, *cfg, out);
  else
    hipLaunchKernelGGL(grid_obs_kernel<float>, dim3(s->n_envs), dim3(nt), lds, st, *s, *road, *p, *cfg, out);
  return launch_status();
}

int ttrl_observe_ttc(const ttrl_state_t* s, const ttrl_lane_table_t* road, const ttrl_params_t* p,
                     const ttrl_ttc_cfg_t* cfg, float* out, void* stream) {
  int rc = check_state(s, road);
  if (rc) return rc < 0 ? rc : TTRL_OK;
  const bool raw = cfg && cfg->obs_lanes == 0 && cfg->obs_speeds == 0;
  if (!p || !cfg || !out || cfg->horizon_bins < 1 || cfg->horizon_bins > 64 || (!raw && cfg->obs_lanes < 1) ||
      (!raw && cfg->obs_speeds < 1) || !(cfg->time_quantization > 0) || p->n_target_speeds < 1 ||
      p->n_target_speeds > 8)
    return TTRL_E_ARG;
  if (s->n_envs == 0) return TTRL_OK;
  const size_t lds = sizeof(int) * p->n_target_speeds * road->n_lanes * cfg->horizon_bins;
  hipStream_t st = (hipStream_t)stream;
  if (s->dtype == TTRL_F64)
    hipLaunchKernelGGL(ttc_obs_kernel<double>, dim3(s->n_envs), dim3(64), lds, st, *s, *road, *p, *cfg, out);
  else
    hipLaunchKernelGGL(ttc_obs_kernel<float>, dim3(s->n_envs), dim3(64), lds, st, *s, *road, *p, *cfg, out);
  return launch_status();
}

int ttrl_observe_lidar(const ttrl_state_t* s, const ttrl_lane_table_t* road, const ttrl_params_t* p,
                       const ttrl_lidar_cfg_t* cfg, float* out, void* stream) {
  int rc = check_state(s, road);
  if (rc) return rc < 0 ? rc : TTRL_OK;
  if (!p || !cfg || !out || cfg->cells < 1 || cfg->cells > 64 || !(cfg->maximum_range > 0)) return TTRL_E_ARG;
  if (s->n_envs == 0) return TTRL_OK;
  hipStream_t st = (hipStream_t)stream;
  if (s->dtype == TTRL_F64)
    hipLaunchKernelGGL(lidar_obs_kernel<double>, dim3(s->n_envs), dim3(64), 0, st, *s, *p, *cfg, out);
  else
    hipLaunchKernelGGL(lidar_obs_kernel<float>, dim3(s->n_envs), dim3(64), 0, st, *s, *p, *cfg, out);
  return launch_status();
}

int ttrl_reset_highway(const ttrl_state_t* s, const ttrl_lane_table_t* road, const ttrl_params_t* p,
                       const ttrl_reset_cfg_t* cfg, const uint64_t* pcg, void* stream) {
  int rc = check_state(s, road);
  if (rc) return rc < 0 ? rc : TTRL_OK;
  if (!p || !cfg || !pcg || cfg->n_vehicles < 1 || cfg->n_vehicles > s->n_veh || cfg->ego_lane < 0 ||
      cfg->ego_lane >= road->n_lanes || p->n_target_speeds < 1 || p->n_target_speeds > 8)
    return TTRL_E_ARG;
  if (s->n_envs == 0) return TTRL_OK;
  hipStream_t st = (hipStream_t)stream;
  if (s->dtype == TTRL_F64)
    launch_reset<double>(*s, *road, *p, *cfg, (const unsigned long long*)pcg, nullptr, 0, nullptr, AutoReset{}, st);
  else
    launch_reset<float>(*s, *road, *p, *cfg, (const unsigned long long*)pcg, nullptr, 0, nullptr, AutoReset{}, st);
  return launch_status();
}

int ttrl_reset_highway_seeded(const ttrl_state_t* s, const ttrl_lane_table_t* road, const ttrl_params_t* p,
                              const ttrl_reset_cfg_t* cfg, const uint32_t* entropy, int32_t n_words,
                              const uint8_t* mask, void* stream) {
  int rc = check_state(s, road);
  if (rc) return rc < 0 ? rc : TTRL_OK;
  if (!p || !cfg || !entropy || n_words < 1 || n_words > 64 || cfg->n_vehicles < 1 || cfg->n_vehicles > s->n_veh ||
      cfg->ego_lane < 0 || cfg->ego_lane >= road->n_lanes || p->n_target_speeds < 1 || p->n_target_speeds > 8)
    return TTRL_E_ARG;
  if (s->n_envs == 0) return TTRL_OK;
  hipStream_t st = (hipStream_t)stream;
  if (s->dtype == TTRL_F64)
    launch_reset<double>(*s, *road, *p, *cfg, nullptr, (unsigned*)entropy, (int)n_words, mask, AutoReset{}, st);
  else
    launch_reset<float>(*s, *road, *p, *cfg, nullptr, (unsigned*)entropy, (int)n_words, mask, AutoReset{}, st);
  return launch_status();
}

int ttrl_auto_reset_highway(const ttrl_state_t* s, const ttrl_lane_table_t* road, const ttrl_params_t* p,
                            const ttrl_reset_cfg_t* cfg, uint32_t* entropy, int32_t n_words, int32_t episode_word,
                            const uint8_t* terminated, const uint8_t* truncated, double* time, uint8_t* done,
                            void* stream) {
  int rc = check_state(s, road);
  if (rc) return rc < 0 ? rc : TTRL_OK;
  if (!p || !cfg || !entropy || !terminated || !truncated || !time || !done || n_words < 1 || n_words > 8 ||
      episode_word < 0 || episode_word >= n_words || cfg->n_vehicles < 1 || cfg->n_vehicles > s->n_veh ||
      cfg->ego_lane < 0 || cfg->ego_lane >= road->n_lanes || p->n_target_speeds < 1 || p->n_target_speeds > 8)
    return TTRL_E_ARG;
  if (s->n_envs == 0) return TTRL_OK;
  hipStream_t st = (hipStream_t)stream;
  const AutoReset ar{terminated, truncated, time, done, episode_word};
  if (s->dtype == TTRL_F64)
    launch_reset<double>(*s, *road, *p, *cfg, nullptr, (unsigned*)entropy, (int)n_words, nullptr, ar, st);
  else
    launch_reset<float>(*s, *road, *p, *cfg, nullptr, (unsigned*)entropy, (int)n_words, nullptr, ar, st);
  return launch_status();
}

int ttrl_seed_pcg64(const uint32_t* entropy, int32_t n_words, uint64_t* state4) {
  if (!entropy || !state4 || n_words < 1 || n_words > 64) return TTRL_E_ARG;
  unsigned long long o[4];
  SeedSeq::pcg64_seed((const unsigned*)entropy, n_words, o);
  for (int k = 0; k < 4; ++k) state4[k] = o[k];
  return TTRL_OK;
}

static int check_ix(const ttrl_state_t* s, const ttrl_lane_table_t* R, const ttrl_params_t* p, const ttrl_ix_cfg_t* c) {
  int rc = check_state(s, R);
  if (rc) return rc;  // EMPTY propagates
  if (!p || !c || !s->rng || !s->route_road || !s->route_lane || !s->route_n || !s->yielding || !s->reg_steps)
    return TTRL_E_ARG;
  if (p->n_target_speeds < 1 || p->n_target_speeds > 8 || c->n_corners != 4) return TTRL_E_ARG;
  if (c->initial_vehicle_count < 1 || c->initial_vehicle_count > TTRL_IX_MAX_INIT || c->warmup_frames < 0)
    return TTRL_E_ARG;
  if (c->ego_lane < 0 || c->ego_lane >= R->n_lanes || c->ego_destination < -1 || c->ego_destination > 3) return TTRL_E_ARG;
  for (int k = 0; k < 4; ++k)
    if (c->entry_lane[k] < 0 || c->entry_lane[k] >= R->n_lanes) return TTRL_E_ARG;
  for (int r = 0; r < R->n_roads; ++r)
    if (R->road_from[r] < 0 || R->road_from[r] >= TTRL_MAX_NODES || R->road_to[r] < 0 || R->road_to[r] >= TTRL_MAX_NODES)
      return TTRL_E_ARG;
  for (int nd = 0; nd < TTRL_MAX_NODES; ++nd)
    for (int k = 0; k < 4; ++k) {
      if (c->path_len[nd][k] > TTRL_ROUTE_MAX - 1) return TTRL_E_ARG;
      for (int q = 0; q < c->path_len[nd][k]; ++q)
        if (c->path_road[nd][k][q] < 0 || c->path_road[nd][k][q] >= R->n_roads) return TTRL_E_ARG;
    }
  return TTRL_OK;
}

int ttrl_ix_reset_parts(const ttrl_state_t* s, const ttrl_lane_table_t* road, const ttrl_params_t* p,
                        const ttrl_ix_cfg_t* cfg, int32_t parts, const uint32_t* entropy, int32_t n_words,
                        const uint8_t* begin_mask, const uint8_t* warm_mask, int32_t warm_frames,
                        const uint8_t* finish_mask, void* stream) {
  int rc = check_ix(s, road, p, cfg);
  if (rc) return rc < 0 ? rc : TTRL_OK;
  if (parts < 0 || parts > 7 || warm_frames < 0) return TTRL_E_ARG;
  if ((parts & TTRL_IX_BEGIN) && (!entropy || n_words < 1 || n_words > 64)) return TTRL_E_ARG;
  if (s->n_envs == 0) return TTRL_OK;
  hipStream_t st = (hipStream_t)stream;
  const int blocks = s->n_envs;  // one wavefront per env
  if (parts & TTRL_IX_BEGIN) {
    if (s->dtype == TTRL_F64)
      hipLaunchKernelGGL(ix_begin_kernel<double>, dim3(blocks), dim3(64), 0, st, *s, *road, *p, *cfg,
                         (const unsigned*)entropy, (int)n_words, begin_mask);
    else
      hipLaunchKernelGGL(ix_begin_kernel<float>, dim3(blocks), dim3(64), 0, st, *s, *road, *p, *cfg,
                         (const unsigned*)entropy, (int)n_words, begin_mask);
    if ((rc = launch_status())) return rc;
  }
  // _make_vehicles' warm-up: 3 s of Road.act / Road.step with no controlled vehicle yet; frames
  // [f, f + n) then [f + n, ...) equal [f, ...) in one launch (the state round-trips HBM exactly)
  if ((parts & TTRL_IX_WARMUP) && warm_frames > 0 &&
      (rc = run_sim(s, road, p, nullptr, warm_frames, cfg->warmup_dt, MODE_ACT | MODE_STEP, stream, 0, warm_mask)))
    return rc;
  if (parts & TTRL_IX_FINISH) {
    if (s->dtype == TTRL_F64)
      hipLaunchKernelGGL(ix_finish_kernel<double>, dim3(blocks), dim3(64), 0, st, *s, *road, *p, *cfg, finish_mask);
    else
      hipLaunchKernelGGL(ix_finish_kernel<float>, dim3(blocks), dim3(64), 0, st, *s, *road, *p, *cfg, finish_mask);
  }
  return launch_status();
}

int ttrl_ix_reset(const ttrl_state_t* s, const ttrl_lane_table_t* road, const ttrl_params_t* p,
                  const ttrl_ix_cfg_t* cfg, const uint32_t* entropy, int32_t n_words, const uint8_t* mask,
                  void* stream) {
  if (!cfg) return TTRL_E_ARG;
  return ttrl_ix_reset_parts(s, road, p, cfg, TTRL_IX_BEGIN | TTRL_IX_WARMUP | TTRL_IX_FINISH, entropy, n_words,
                             mask, mask, cfg->warmup_frames, mask, stream);
}

int ttrl_copy_envs(const ttrl_state_t* dst, const ttrl_state_t* src, const uint8_t* mask, void* stream) {
  if (!dst || !src || !mask) return TTRL_E_ARG;
  if (dst->n_envs != src->n_envs || dst->n_veh != src->n_veh || dst->dtype != src->dtype) return TTRL_E_ARG;
  if (dst->n_envs < 0 || dst->n_veh < 1 || dst->n_veh > 256 || (dst->dtype != TTRL_F32 && dst->dtype != TTRL_F64))
    return TTRL_E_ARG;
  if (dst->n_envs == 0) return TTRL_OK;
  const void* ptrs[] = {dst->x, dst->y, dst->heading, dst->speed, dst->target_speed, dst->timer, dst->delta, dst->steer,
                        dst->acc, dst->impact_x, dst->impact_y, dst->lane, dst->target_lane, dst->speed_index,
                        dst->kind, dst->crashed, dst->has_impact, dst->lane_change, src->x, src->y, src->heading,
                        src->speed, src->target_speed, src->timer, src->delta, src->steer, src->acc, src->impact_x,
                        src->impact_y, src->lane, src->target_lane, src->speed_index, src->kind, src->crashed,
                        src->has_impact, src->lane_change};
  for (const void* q : ptrs)
    if (!q) return TTRL_E_ARG;
  if ((dst->route_road != nullptr) != (src->route_road != nullptr)) return TTRL_E_ARG;
  if (dst->route_road && (!dst->route_lane || !dst->route_n || !dst->yielding || !src->route_lane || !src->route_n ||
                          !src->yielding))
    return TTRL_E_ARG;
  hipStream_t st = (hipStream_t)stream;
  if (dst->dtype == TTRL_F64)
    hipLaunchKernelGGL(copy_envs_kernel<double>, dim3(dst->n_envs), dim3(64), 0, st, *dst, *src, mask);
  else
    hipLaunchKernelGGL(copy_envs_kernel<float>, dim3(dst->n_envs), dim3(64), 0, st, *dst, *src, mask);
  return launch_status();
}

int ttrl_ix_clear_spawn(const ttrl_state_t* s, const ttrl_lane_table_t* road, const ttrl_params_t* p,
                        const ttrl_ix_cfg_t* cfg, const uint8_t* mask, void* stream) {
  int rc = check_ix(s, road, p, cfg);
  if (rc) return rc < 0 ? rc : TTRL_OK;
  if (s->n_envs == 0) return TTRL_OK;
  hipStream_t st = (hipStream_t)stream;
  const int blocks = s->n_envs;  // one wavefront per env
  if (s->dtype == TTRL_F64)
    hipLaunchKernelGGL(ix_clear_spawn_kernel<double>, dim3(blocks), dim3(64), 0, st, *s, *road, *p, *cfg, mask);
  else
    hipLaunchKernelGGL(ix_clear_spawn_kernel<float>, dim3(blocks), dim3(64), 0, st, *s, *road, *p, *cfg, mask);
  return launch_status();
}

int ttrl_ix_step_tail(const ttrl_state_t* s, const ttrl_lane_table_t* road, const ttrl_params_t* p,
                      const ttrl_ix_cfg_t* cfg, const ttrl_state_t* spare, const uint8_t* terminated,
                      const uint8_t* truncated, uint8_t* spare_parity, uint32_t* entropy, uint32_t* spare_entropy,
                      int32_t n_words, double* time, uint8_t* done, uint8_t* spare_mask,
                      const ttrl_kin_cfg_t* obs_cfg, const float* obs_in, float* obs_out, const int32_t* obs_ids_in,
                      int32_t* obs_ids_out, int64_t* live_count, int32_t* order, void* stream) {
  int rc = check_ix(s, road, p, cfg);
  if (rc) return rc < 0 ? rc : TTRL_OK;
  if (!spare || !terminated || !truncated || !spare_parity || !entropy || !spare_entropy || n_words < 1 ||
      n_words > 65 || !time || !done || !spare_mask)
    return TTRL_E_ARG;
  const int K = s->n_envs > 0 ? spare->n_envs / s->n_envs : 0;
  if (K < 2 || K > 16 || spare->n_envs != K * s->n_envs || spare->n_veh != s->n_veh || spare->dtype != s->dtype || !spare->rng ||
      !spare->reg_steps || !spare->route_road || !spare->route_lane || !spare->route_n || !spare->yielding)
    return TTRL_E_ARG;
  const void* sp[] = {spare->x, spare->y, spare->heading, spare->speed, spare->target_speed, spare->timer,
                      spare->delta, spare->steer, spare->acc, spare->impact_x, spare->impact_y, spare->lane,
                      spare->target_lane, spare->speed_index, spare->kind, spare->crashed, spare->has_impact,
                      spare->lane_change};
  for (const void* q : sp)
    if (!q) return TTRL_E_ARG;
  if (obs_cfg) {  // the re-observation puts one slot on each lane of the env's wavefront
    if (check_kin_cfg(s, obs_cfg) || !obs_in || !obs_out || (!obs_ids_in) != (!obs_ids_out) || s->n_veh > 64)
      return obs_cfg && s->n_veh > 64 ? TTRL_E_UNSUPPORTED : TTRL_E_ARG;
  }
  IxTail t{};
  t.spare = *spare; t.K = K; t.term = terminated; t.trunc = truncated; t.par = spare_parity; t.ent = entropy;
  t.spare_ent = spare_entropy; t.nw = n_words; t.time = time; t.done = done; t.spare_mask = spare_mask;
  t.live = reinterpret_cast<unsigned long long*>(live_count);
  // the dispatch order groups the envs of one simulate workgroup (EPW: 2 on 32 slots, else 1)
  const int G = slots_for(s->n_veh) == 32 ? 2 : 1;
  const bool ordered = order && s->n_envs % G == 0;
  if (ordered) t.live_env = order + s->n_envs;
  if (obs_cfg) {
    t.kcfg = *obs_cfg; t.obs = true; t.obs_in = obs_in; t.obs_out = obs_out; t.ids_in = obs_ids_in;
    t.ids_out = obs_ids_out;
  }
  hipStream_t st = (hipStream_t)stream;
  if (s->dtype == TTRL_F64)
    hipLaunchKernelGGL(ix_step_tail_kernel<double>, dim3(s->n_envs), dim3(64), 0, st, *s, *road, *p, *cfg, t);
  else
    hipLaunchKernelGGL(ix_step_tail_kernel<float>, dim3(s->n_envs), dim3(64), 0, st, *s, *road, *p, *cfg, t);
  if (ordered)
    hipLaunchKernelGGL(ix_order_kernel, dim3(1), dim3(1024), 0, st, order, s->n_envs, G, G * s->n_veh);
  return launch_status();
}

int ttrl_ix_env_step(const ttrl_state_t* s, const ttrl_lane_table_t* road, const ttrl_params_t* p,
                     const ttrl_ix_cfg_t* cfg, const int32_t* actions, int32_t frames, double dt,
                     const ttrl_kin_cfg_t* obs_cfg, float* obs, int32_t* obs_ids, float* obs_next, int32_t* ids_next,
                     const ttrl_reward_cfg_t* reward_cfg, double* time, double time_inc, float* reward,
                     uint8_t* terminated, uint8_t* truncated, float* components, void* ego_speed,
                     uint8_t* ego_crashed, const ttrl_state_t* spare, uint8_t* spare_parity, uint32_t* entropy,
                     uint32_t* spare_entropy, int32_t n_words, uint8_t* done, uint8_t* spare_mask, int32_t* order,
                     const int32_t* action_lut, int32_t n_action_lut, int64_t* live_count, void* stream) {
  int rc = check_ix(s, road, p, cfg);
  if (rc) return rc < 0 ? rc : TTRL_OK;
  if (!spare || !spare_parity || !entropy || !spare_entropy || n_words < 1 || n_words > 65 || !done || !spare_mask)
    return TTRL_E_ARG;
  const int K = spare->n_envs / s->n_envs;
  if (K < 2 || K > 16 || spare->n_envs != K * s->n_envs || spare->n_veh != s->n_veh || spare->dtype != s->dtype ||
      !spare->rng || !spare->reg_steps || !spare->route_road || !spare->route_lane || !spare->route_n || !spare->yielding)
    return TTRL_E_ARG;
  {
    const void* sp[] = {spare->x, spare->y, spare->heading, spare->speed, spare->target_speed, spare->timer,
                        spare->delta, spare->steer, spare->acc, spare->impact_x, spare->impact_y, spare->lane,
                        spare->target_lane, spare->speed_index, spare->kind, spare->crashed, spare->has_impact,
                        spare->lane_change};
    for (const void* q : sp)
      if (!q) return TTRL_E_ARG;
  }
  if (!obs_cfg || !obs || !obs_next || check_kin_cfg(s, obs_cfg) || (!obs_ids) != (!ids_next)) return TTRL_E_ARG;
  if (!reward_cfg || !time || !reward || !terminated || !truncated || (!ego_speed) != (!ego_crashed))
    return TTRL_E_ARG;
  if (n_action_lut < 0 || n_action_lut > 8 || (n_action_lut > 0 && !action_lut)) return TTRL_E_ARG;
  if (slots_for(s->n_veh) > 64) return TTRL_E_UNSUPPORTED;  // the fused tail needs one wavefront per workgroup
  StepOut so{};
  for (int q = 0; q < n_action_lut; ++q) {
    if (action_lut[q] < TTRL_LANE_LEFT || action_lut[q] > TTRL_SLOWER) return TTRL_E_ARG;
    so.lut[q] = (int8_t)action_lut[q];
  }
  so.n_lut = n_action_lut;
  so.kcfg = *obs_cfg; so.obs = obs; so.ids = obs_ids;
  so.rcfg = *reward_cfg; so.time = time; so.time_inc = time_inc; so.reward = reward; so.term = terminated;
  so.trunc = truncated; so.comp = components; so.ego_speed = ego_speed; so.ego_crashed = ego_crashed;
  so.order = order;
  IxEpi ie{};
  ie.C = *cfg;
  ie.lane_change_delay = p->lane_change_delay;
  ie.obs2 = obs_next; ie.ids2 = ids_next;
  ie.live = reinterpret_cast<unsigned long long*>(live_count);
  ie.spare = *spare; ie.K = K; ie.par = spare_parity; ie.ent = entropy; ie.spare_ent = spare_entropy;
  ie.nw = n_words; ie.done = done; ie.spare_mask = spare_mask;
  const int G = slots_for(s->n_veh) == 32 ? 2 : 1;  // envs per wavefront (the dispatch order's groups)
  const bool ordered = order && s->n_envs % G == 0;
  if (ordered) ie.live_env = order + s->n_envs;  // ix_order_kernel's input
  hipStream_t st = (hipStream_t)stream;
  if (s->dtype == TTRL_F64)
    rc = G == 2 ? launch_sim_ix<double, 32, 2>(*s, *road, *p, actions, frames, dt, st, so, ie)
                : launch_sim_ix<double, 64, 1>(*s, *road, *p, actions, frames, dt, st, so, ie);
  else
    rc = G == 2 ? launch_sim_ix<float, 32, 2>(*s, *road, *p, actions, frames, dt, st, so, ie)
                : launch_sim_ix<float, 64, 1>(*s, *road, *p, actions, frames, dt, st, so, ie);
  if (rc) return rc;
  if (ordered)  // the next step's dispatch order, as ttrl_ix_step_tail writes it
    hipLaunchKernelGGL(ix_order_kernel, dim3(1), dim3(1024), 0, st, order, s->n_envs, G, G * s->n_veh);
  return launch_status();
}

int ttrl_rewards_step(const ttrl_state_t* s, const ttrl_lane_table_t* road, const ttrl_reward_cfg_t* cfg,
                      double* time, double time_inc, float* reward, uint8_t* terminated, uint8_t* truncated,
                      float* components, void* ego_speed, uint8_t* ego_crashed, void* stream) {
  int rc = check_state(s, road);
  if (rc) return rc < 0 ? rc : TTRL_OK;
  if (!cfg || !time || !reward || !terminated || !truncated || (!ego_speed) != (!ego_crashed)) return TTRL_E_ARG;
  hipStream_t st = (hipStream_t)stream;
  const int blocks = (s->n_envs + 255) / 256;
  if (s->dtype == TTRL_F64)
    hipLaunchKernelGGL(rewards_kernel<double>, dim3(blocks), dim3(256), 0, st, *s, *road, *cfg, time, time_inc,
                       reward, terminated, truncated, components, (double*)ego_speed, ego_crashed);
  else
    hipLaunchKernelGGL(rewards_kernel<float>, dim3(blocks), dim3(256), 0, st, *s, *road, *cfg, time, time_inc,
                       reward, terminated, truncated, components, (float*)ego_speed, ego_crashed);
  return launch_status();
}

int ttrl_rewards_ex(const ttrl_state_t* s, const ttrl_lane_table_t* road, const ttrl_reward_cfg_t* cfg,
                    const double* time, float* reward, uint8_t* terminated, uint8_t* truncated, float* components,
                    void* stream) {
  // time_inc 0: the kernel only reads time
  return ttrl_rewards_step(s, road, cfg, const_cast<double*>(time), 0.0, reward, terminated, truncated, components,
                           nullptr, nullptr, stream);
}

int ttrl_rewards(const ttrl_state_t* s, const ttrl_lane_table_t* road, const ttrl_reward_cfg_t* cfg,
                 const double* time, float* reward, uint8_t* terminated, uint8_t* truncated, void* stream) {
  return ttrl_rewards_ex(s, road, cfg, time, reward, terminated, truncated, nullptr, stream);
}

}  // extern "C"
#endif  // TTRL_KERNEL_ONLY
