/*
 * ttrl_oracle.c — TEST INFRASTRUCTURE ONLY (parity checker, CPU baseline).
 *
 * A plain-C, float64, strictly sequential restatement of the reference's
 * env.step() hot path (ITCAAdvancedTeam/TopoTrafficRL, ttrl_env).  Each function
 * follows one reference function and cites it; loops run in the reference's
 * list order so Gauss-Seidel reads (change_lane_policy) and last-writer
 * collision impacts come out exactly as in Python.  Compiled with
 * -ffp-contract=off so every + and * rounds like numpy float64.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline call this.
 * The product path (topotrafficrl_amd) never links or loads it.
 *
 * Pinned against tests/golden/ (npz files), which oracle/gen_golden.py captures from
 * the unmodified reference sim core.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/ttrl_mi355x.h"

typedef struct {
  int E, N;
  double *x, *y, *h, *v, *ts, *timer, *delta, *steer, *acc, *ix, *iy;
  int32_t *lane, *tgt, *sidx;
  uint8_t *kind, *crashed, *hasimp, *lc;
  int8_t *rroad, *rlane, *rn;   /* route entries [E*N][TTRL_ROUTE_MAX], length (-1 = None) */
  uint8_t* yield;
  int32_t* reg;
  uint64_t* rng;                /* [E][TTRL_RNG_WORDS] np_random */
  double* mg;                   /* [E*N] decision margins (oracle_frame_margins), NULL otherwise */
  int32_t* mgsite;              /* [E*N] source line of each vehicle's smallest margin */
  int32_t* lk;                  /* [E*N][lkmax] causal links (oracle_frame_links), NULL otherwise */
  int lkmax;
} S;

static S view(const ttrl_state_t* s) {
  S o;
  o.E = s->n_envs; o.N = s->n_veh;
  o.x = (double*)s->x; o.y = (double*)s->y; o.h = (double*)s->heading; o.v = (double*)s->speed;
  o.ts = (double*)s->target_speed; o.timer = (double*)s->timer; o.delta = (double*)s->delta;
  o.steer = (double*)s->steer; o.acc = (double*)s->acc; o.ix = (double*)s->impact_x; o.iy = (double*)s->impact_y;
  o.lane = s->lane; o.tgt = s->target_lane; o.sidx = s->speed_index;
  o.kind = s->kind; o.crashed = s->crashed; o.hasimp = s->has_impact; o.lc = s->lane_change;
  o.rroad = s->route_road; o.rlane = s->route_lane; o.rn = s->route_n; o.yield = s->yielding; o.reg = s->reg_steps;
  o.rng = s->rng;
  o.mg = NULL; o.mgsite = NULL; o.lk = NULL; o.lkmax = 0;
  return o;
}

/* Decision margins (oracle_frame_margins only): every comparison whose outcome is discrete
 * (a threshold, an argmin, a tie-break) records |distance to the switch point| / (1 + |scale|)
 * for the vehicle it decides for, keeping the minimum.  A float32 result may legitimately flip
 * such a decision only where this float64 margin is below the float32 working precision. */
static void mg_at(const S* o, int k, double m, double scale, int line) {
  if (!o->mg) return;
  double r = fabs(m) / (1.0 + fabs(scale));
  if (r < o->mg[k]) { o->mg[k] = r; if (o->mgsite) o->mgsite[k] = line; }
}
#define mg(o, k, m, scale) mg_at(o, k, m, scale, __LINE__)

/* Causal links (oracle_frame_links only): within one frame, vehicle k's discrete outcomes read
 * another vehicle j's results of the SAME frame in two places only -- the lane-change abort reads
 * the targets that vehicles earlier in the list set this frame (behavior.py:229-244), and the
 * collision pass reads every vehicle's post-step pose (objects.py:91-137).  Every j whose changed
 * result could change k's outcome there is recorded in k's row (slots within the env, -1 padded;
 * a full row ends in -2).  Reads of frame-start state (neighbour scans, MOBIL, IDM) are not links:
 * both precisions start the frame from the same inputs. */
static void link_at(const S* o, int k, int j) {
  if (!o->lk) return;
  int32_t* row = o->lk + (size_t)k * o->lkmax;
  for (int q = 0; q < o->lkmax; ++q) {
    if (row[q] == j) return;
    if (row[q] == -1) { row[q] = j; return; }
  }
  row[o->lkmax - 1] = -2;
}

static const double PI = 3.141592653589793;

/* utils.py:48-54 */
static double not_zero(double x) {
  const double eps = 1e-2;
  if (fabs(x) > eps) return x;
  return x >= 0 ? eps : -eps;
}
/* numpy float64 remainder (sign of divisor) */
static double pymod(double a, double b) {
  double m = fmod(a, b);
  if (m != 0.0) { if ((b < 0) != (m < 0)) m += b; }
  else m = copysign(0.0, b);
  return m;
}
/* utils.py:57-58 */
static double wrap_to_pi(double x) { return pymod(x + PI, 2 * PI) - PI; }
static double clipd(double x, double lo, double hi) { return x < lo ? lo : (x > hi ? hi : x); }
/* utils.py:29-31 */
static double lmap(double v, double x0, double x1, double y0, double y1) {
  return y0 + (v - x0) * (y1 - y0) / (x1 - x0);
}

/* local_coordinates: StraightLane lane.py:209-213 (np.dot of 2-vectors), SineLane :275-279,
 * CircularLane :327-334 */
/* numpy PCG64 (pcg_setseq_128_xsl_rr_64): step, then output of the new state. */
typedef struct { unsigned __int128 st, inc; int has32; uint32_t u32; } pcg_t;
static const unsigned __int128 PCG_MULT =
    ((unsigned __int128)0x2360ED051FC65DA4ULL << 64) | 0x4385DF649FCCF645ULL;
static uint64_t pcg_next64(pcg_t* g) {
  g->st = g->st * PCG_MULT + g->inc;
  uint64_t hi = (uint64_t)(g->st >> 64), lo = (uint64_t)g->st;
  uint64_t x = hi ^ lo; unsigned rot = (unsigned)(hi >> 58);
  return (x >> rot) | (x << ((64 - rot) & 63));
}
static uint32_t pcg_next32(pcg_t* g) {
  if (g->has32) { g->has32 = 0; return g->u32; }
  uint64_t n = pcg_next64(g); g->has32 = 1; g->u32 = (uint32_t)(n >> 32); return (uint32_t)n;
}
static double pcg_double(pcg_t* g) { return (double)(pcg_next64(g) >> 11) * (1.0 / 9007199254740992.0); }
/* Generator.integers(0, n) for 1 < n <= 2^32 (buffered Lemire, numpy distributions.c) */
static uint32_t pcg_bounded(pcg_t* g, uint32_t n) {
  if (n <= 1) return 0;
  uint32_t rng = n - 1; uint64_t rexcl = (uint64_t)rng + 1;
  uint64_t m = (uint64_t)pcg_next32(g) * rexcl;
  uint32_t left = (uint32_t)m;
  if (left < rexcl) {
    uint32_t thr = (uint32_t)((0xFFFFFFFFULL - rng) % rexcl);
    while (left < thr) { m = (uint64_t)pcg_next32(g) * rexcl; left = (uint32_t)m; }
  }
  return (uint32_t)(m >> 32);
}
static double pcg_uniform(pcg_t* g, double lo, double hi) { return lo + (hi - lo) * pcg_double(g); }


/* ---- numpy.random.Generator over PCG64, restated (numpy 1.26 / 2.2 random/src/distributions/
 * distributions.c and _generator.pyx; the reference draws through gymnasium's np_random,
 * seeding.np_random = Generator(PCG64(SeedSequence(seed)))).  Pinned against numpy itself by
 * tests/test_ix_rng.py. */
static void rng_load(pcg_t* g, const uint64_t* w) {
  g->st = ((unsigned __int128)w[0] << 64) | w[1];
  g->inc = ((unsigned __int128)w[2] << 64) | w[3];
  g->has32 = (int)(w[4] >> 32); g->u32 = (uint32_t)w[4];
}
static void rng_store(const pcg_t* g, uint64_t* w) {
  w[0] = (uint64_t)(g->st >> 64); w[1] = (uint64_t)g->st;
  w[2] = (uint64_t)(g->inc >> 64); w[3] = (uint64_t)g->inc;
  w[4] = ((uint64_t)(g->has32 ? 1 : 0) << 32) | g->u32;
}
/* random_interval: uniform on [0, max] by masked rejection (Generator.shuffle) */
static uint64_t pcg_interval(pcg_t* g, uint64_t max) {
  if (max == 0) return 0;
  uint64_t mask = max, v;
  mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16; mask |= mask >> 32;
  if (max <= 0xffffffffULL) { while ((v = (pcg_next32(g) & mask)) > max) {} }
  else { while ((v = (pcg_next64(g) & mask)) > max) {} }
  return v;
}
#include "../topotrafficrl_amd/csrc/ttrl_ziggurat.h"
/* random_standard_normal: 256-entry ziggurat (ziggurat_constants.h) */
static double pcg_normal(pcg_t* g) {
  for (;;) {
    uint64_t r = pcg_next64(g);
    const int idx = (int)(r & 0xff);
    r >>= 8;
    const int sign = (int)(r & 0x1);
    const uint64_t rabs = (r >> 1) & 0x000fffffffffffffULL;
    double x = (double)rabs * ttrl_zig_wi[idx];
    if (sign & 0x1) x = -x;
    if (rabs < ttrl_zig_ki[idx]) return x;
    if (idx == 0) {
      for (;;) {
        const double xx = -TTRL_ZIG_NOR_INV_R * log1p(-pcg_double(g));
        const double yy = -log1p(-pcg_double(g));
        if (yy + yy > xx * xx) return ((rabs >> 8) & 0x1) ? -(TTRL_ZIG_NOR_R + xx) : TTRL_ZIG_NOR_R + xx;
      }
    } else {
      if (((ttrl_zig_fi[idx - 1] - ttrl_zig_fi[idx]) * pcg_double(g) + ttrl_zig_fi[idx]) < exp(-0.5 * x * x))
        return x;
    }
  }
}
/* Generator.choice(pop, size, replace=False) for a small population: Floyd's algorithm, then
 * _shuffle_int (random_bounded_uint64 draws) */
static void pcg_choice_noreplace(pcg_t* g, int pop, int size, int* out) {
  for (int j = pop - size; j < pop; ++j) {
    const int val = (int)pcg_bounded(g, (uint32_t)j + 1);
    int seen = 0;
    for (int q = 0; q < j - (pop - size); ++q) seen |= out[q] == val;
    out[j - (pop - size)] = seen ? j : val;
  }
  for (int i = size - 1; i >= 1; --i) {
    const int j = (int)pcg_bounded(g, (uint32_t)i + 1);
    const int t = out[i]; out[i] = out[j]; out[j] = t;
  }
}

static void local(const ttrl_lane_table_t* R, int l, double px, double py, double* s, double* r) {
  if (R->type[l] == TTRL_LANE_CIRCULAR) {
    double dx = px - R->center_x[l], dy = py - R->center_y[l];
    double phi = atan2(dy, dx);
    phi = R->start_phase[l] + wrap_to_pi(phi - R->start_phase[l]);
    double rr = sqrt(dx * dx + dy * dy);
    *s = R->direction[l] * (phi - R->start_phase[l]) * R->radius[l];
    *r = R->direction[l] * (R->radius[l] - rr);
    return;
  }
  double dx = px - R->start_x[l], dy = py - R->start_y[l];
  *s = dx * R->dir_x[l] + dy * R->dir_y[l];
  *r = dx * (-R->dir_y[l]) + dy * R->dir_x[l];
  if (R->type[l] == TTRL_LANE_SINE) *r = *r - R->amplitude[l] * sin(R->pulsation[l] * *s + R->phase[l]);
}
/* heading_at: StraightLane :197-198, SineLane :269-273, CircularLane :318-321 */
static double heading_at(const ttrl_lane_table_t* R, int l, double s) {
  if (R->type[l] == TTRL_LANE_SINE)
    return R->heading[l] + atan(R->amplitude[l] * R->pulsation[l] * cos(R->pulsation[l] * s + R->phase[l]));
  if (R->type[l] == TTRL_LANE_CIRCULAR) {
    double phi = R->direction[l] * s / R->radius[l] + R->start_phase[l];
    return phi + PI / 2 * R->direction[l];
  }
  return R->heading[l];
}
/* position: StraightLane :199-204, SineLane :263-267, CircularLane :313-316 */
static void position(const ttrl_lane_table_t* R, int l, double s, double r, double* x, double* y) {
  if (R->type[l] == TTRL_LANE_CIRCULAR) {
    double phi = R->direction[l] * s / R->radius[l] + R->start_phase[l];
    double k = R->radius[l] - r * R->direction[l];
    *x = R->center_x[l] + k * cos(phi);
    *y = R->center_y[l] + k * sin(phi);
    return;
  }
  if (R->type[l] == TTRL_LANE_SINE) r = r + R->amplitude[l] * sin(R->pulsation[l] * s + R->phase[l]);
  *x = R->start_x[l] + s * R->dir_x[l] + r * (-R->dir_y[l]);
  *y = R->start_y[l] + s * R->dir_y[l] + r * R->dir_x[l];
}
/* AbstractLane.on_lane lane.py:80-102 */
static int on_lane(const ttrl_lane_table_t* R, const ttrl_params_t* P, int l, double s, double r, double margin) {
  return fabs(r) <= R->width[l] / 2 + margin && -P->lane_vehicle_length <= s && s < R->length[l] + P->lane_vehicle_length;
}
/* AbstractLane.is_reachable_from lane.py:104-118 */
static int reachable(const ttrl_lane_table_t* R, const ttrl_params_t* P, int l, double px, double py) {
  if (R->forbidden[l]) return 0;
  double s, r; local(R, l, px, py, &s, &r);
  return fabs(r) <= 2 * R->width[l] && 0 <= s && s < R->length[l] + P->lane_vehicle_length;
}
/* RoadNetwork.get_closest_lane_index road.py:55-71 + distance_with_heading lane.py:132-147 */
static int closest_lane(const ttrl_lane_table_t* R, double px, double py, double heading) {
  int best = 0; double bd = 0;
  for (int l = 0; l < R->n_lanes; ++l) {
    double s, r; local(R, l, px, py, &s, &r);
    double ang = fabs(wrap_to_pi(heading - heading_at(R, l, s)));
    double a = s - R->length[l]; if (!(a > 0)) a = 0;   /* Python max(s - len, 0) */
    double b = 0 - s; if (!(b > 0)) b = 0;
    double d = fabs(r) + a + b + 1.0 * ang;
    if (l == 0 || d < bd) { bd = d; best = l; }          /* np.argmin: first minimum */
  }
  return best;
}

/* AbstractLane.distance lane.py:127-130 */
static double lane_dist(const ttrl_lane_table_t* R, int l, double px, double py) {
  double s, r; local(R, l, px, py, &s, &r);
  double a = s - R->length[l]; if (0 > a) a = 0;
  double b = 0 - s; if (0 > b) b = 0;
  return fabs(r) + a + b;
}
/* AbstractLane.after_end lane.py:120-125 */
static int after_end(const ttrl_lane_table_t* R, const ttrl_params_t* P, int l, double px, double py) {
  double s, r; local(R, l, px, py, &s, &r);
  return s > R->length[l] - P->lane_vehicle_length / 2;
}
/* RoadNetwork.next_lane_given_next_road road.py:136-154 */
static int next_given(const ttrl_lane_table_t* R, int cur_road, int id, int nroad, int nid, double px, double py,
                      double* dist) {
  if (R->road_n[cur_road] == R->road_n[nroad]) {
    if (nid < 0) nid = id;
  } else {
    double bd = 0;
    for (int l = 0; l < R->road_n[nroad]; ++l) {
      double d = lane_dist(R, R->road_first[nroad] + l, px, py);
      if (l == 0 || d < bd) { bd = d; nid = l; }             /* min(): first minimum */
    }
  }
  *dist = lane_dist(R, R->road_first[nroad] + nid, px, py);
  return nid;
}
/* RoadNetwork.next_lane road.py:73-134, with the route popped in place as in Python */
static int next_lane(S* o, const ttrl_lane_table_t* R, int k, int cur, double x, double y) {
  const int rd = R->road[cur], id = R->lane_id[cur], to = R->road_to[rd];
  int nroad = -1, nid = -1;
  if (o->rn && o->rn[k] > 0) {
    int8_t* rr = o->rroad + (size_t)k * TTRL_ROUTE_MAX;
    int8_t* rl = o->rlane + (size_t)k * TTRL_ROUTE_MAX;
    if (rr[0] == rd) {                                        /* route.pop(0) */
      for (int q = 0; q + 1 < TTRL_ROUTE_MAX; ++q) { rr[q] = rr[q + 1]; rl[q] = rl[q + 1]; }
      rr[TTRL_ROUTE_MAX - 1] = rl[TTRL_ROUTE_MAX - 1] = -1;
      o->rn[k] -= 1;
    }
    if (o->rn[k] > 0 && R->road_from[rr[0]] == to) { nroad = rr[0]; nid = rl[0]; }
  }
  double s, r, px, py;
  local(R, cur, x, y, &s, &r);
  position(R, cur, s, 0, &px, &py);                           /* projected position */
  double d;
  if (nroad < 0) {
    int found = 0; double bd = 0;
    for (int q = 0; q < R->n_roads; ++q) {
      if (R->road_from[q] != to) continue;
      int cand = next_given(R, rd, id, q, -1, px, py, &d);
      if (!found || d < bd) { bd = d; nroad = q; nid = cand; found = 1; }
    }
    if (!found) return cur;                                   /* KeyError: no road leaves `to` */
  } else {
    nid = next_given(R, rd, id, nroad, nid, px, py, &d);
  }
  return R->road_first[nroad] + nid;
}
/* ControlledVehicle.follow_road controller.py:135-143 */
static void follow_road(S* o, const ttrl_lane_table_t* R, const ttrl_params_t* P, int base, int i) {
  const int k = base + i;
  if (o->mg) {
    double s, r; local(R, o->tgt[k], o->x[k], o->y[k], &s, &r);
    mg(o, k, s - (R->length[o->tgt[k]] - P->lane_vehicle_length / 2), s);
  }
  if (after_end(R, P, o->tgt[k], o->x[k], o->y[k])) o->tgt[k] = next_lane(o, R, k, o->tgt[k], o->x[k], o->y[k]);
}

/* RoadObject.lane_distance_to objects.py:182-197 (along `self`'s current lane) */
static double lane_distance(const S* o, const ttrl_lane_table_t* R, int base, int self, int other) {
  int l = o->lane[base + self];
  double s1, r1, s0, r0;
  local(R, l, o->x[base + other], o->y[base + other], &s1, &r1);
  local(R, l, o->x[base + self], o->y[base + self], &s0, &r0);
  return s1 - s0;
}

/* Road.neighbour_vehicles road.py:480-513 */
static void neighbour(const S* o, const ttrl_lane_table_t* R, const ttrl_params_t* P, int base, int self, int l,
                      int* front, int* rear) {
  double s, r; local(R, l, o->x[base + self], o->y[base + self], &s, &r);
  int hf = 0, hr = 0; double sf = 0, sr = 0; *front = *rear = -1;
  for (int j = 0; j < o->N; ++j) {
    if (j == self || o->kind[base + j] == TTRL_ABSENT) continue;
    double sv, lv; local(R, l, o->x[base + j], o->y[base + j], &sv, &lv);
    if (o->mg) {                                                /* on_lane membership, s <= sv */
      mg(o, base + self, fabs(lv) - (R->width[l] / 2 + 1.0), lv);
      mg(o, base + self, sv + P->lane_vehicle_length, sv);
      mg(o, base + self, R->length[l] + P->lane_vehicle_length - sv, sv);
    }
    if (!on_lane(R, P, l, sv, lv, 1.0)) continue;
    if (o->mg) mg(o, base + self, sv - s, s);
    if (s <= sv && (!hf || sv <= sf)) { sf = sv; hf = 1; *front = j; }
    if (sv < s && (!hr || sv > sr)) { sr = sv; hr = 1; *rear = j; }
  }
  if (o->mg && (hf || hr)) {                                    /* runner-up gaps of the two argmins */
    for (int j = 0; j < o->N; ++j) {
      if (j == self || j == *front || j == *rear || o->kind[base + j] == TTRL_ABSENT) continue;
      double sv, lv; local(R, l, o->x[base + j], o->y[base + j], &sv, &lv);
      if (!on_lane(R, P, l, sv, lv, 1.0)) continue;
      if (hf && s <= sv) mg(o, base + self, sv - sf, sf);
      if (hr && sv < s) mg(o, base + self, sr - sv, sr);
    }
  }
}

/* IDMVehicle.desired_gap behavior.py:192-217 (projected=True) */
static double desired_gap(const S* o, const ttrl_params_t* P, int base, int ego, int front) {
  double eh = o->h[base + ego], fh = o->h[base + front], ev = o->v[base + ego], fv = o->v[base + front];
  double ecx = cos(eh), esx = sin(eh);
  double dvx = ev * ecx - fv * cos(fh), dvy = ev * esx - fv * sin(fh);
  double dv = dvx * ecx + dvy * esx;
  return P->distance_wanted + ev * P->time_wanted + ev * dv / P->gap_denom;
}

/* IDMVehicle.acceleration behavior.py:150-190; DELTA is the caller's (`selfd`). */
static double idm_acc(const S* o, const ttrl_lane_table_t* R, const ttrl_params_t* P, int base, double selfd,
                      int ego, int front) {
  if (ego < 0) return 0;
  double ts = o->ts[base + ego];
  ts = clipd(ts, 0, R->speed_limit[o->lane[base + ego]]);
  double v = o->v[base + ego]; if (!(v > 0)) v = (0 > v) ? 0 : v;  /* Python max(v, 0) */
  double a = P->comfort_acc_max * (1 - pow(v / fabs(not_zero(ts)), selfd));
  if (front >= 0) {
    double d = lane_distance(o, R, base, ego, front);
    double q = desired_gap(o, P, base, ego, front) / not_zero(d);
    a -= P->comfort_acc_max * (q * q);
  }
  return a;
}

static int sgn(int x) { return (x > 0) - (x < 0); }
/* IDMVehicle.mobil behavior.py:265-324 */
static int mobil(const S* o, const ttrl_lane_table_t* R, const ttrl_params_t* P, int base, int self, int l) {
  double d = o->delta[base + self];
  int np_, nf; neighbour(o, R, P, base, self, l, &np_, &nf);
  double nfa = idm_acc(o, R, P, base, d, nf, np_);
  double nfpa = idm_acc(o, R, P, base, d, nf, self);
  mg(o, base + self, nfpa + P->lane_change_max_braking, nfpa);
  if (nfpa < -P->lane_change_max_braking) return 0;
  int op, of; neighbour(o, R, P, base, self, o->lane[base + self], &op, &of);
  double spa = idm_acc(o, R, P, base, d, self, np_);
  const int k = base + self;
  if (o->rn && o->rn[k] > 0 && o->rlane[(size_t)k * TTRL_ROUTE_MAX] >= 0) {  /* planned lane (:296-304) */
    const int tid = R->lane_id[o->tgt[k]];
    if (sgn(R->lane_id[l] - tid) != sgn(o->rlane[(size_t)k * TTRL_ROUTE_MAX] - tid)) return 0;
    if (spa < -P->lane_change_max_braking) return 0;
    return 1;
  }
  double sa = idm_acc(o, R, P, base, d, self, op);
  double ofa = idm_acc(o, R, P, base, d, of, self);
  double ofpa = idm_acc(o, R, P, base, d, of, op);
  double jerk = spa - sa + P->politeness * (nfpa - nfa + ofpa - ofa);
  mg(o, base + self, jerk - P->lane_change_min_acc_gain, fabs(spa) + fabs(sa));
  if (jerk < P->lane_change_min_acc_gain) return 0;
  return 1;
}

/* IDMVehicle.change_lane_policy behavior.py:219-263 */
static void change_lane_policy(S* o, const ttrl_lane_table_t* R, const ttrl_params_t* P, int base, int self) {
  int lane = o->lane[base + self], tgt = o->tgt[base + self];
  if (lane != tgt) {
    if (R->road[lane] != R->road[tgt]) return;                 /* not the same road: no abort (:231) */
    for (int j = 0; j < o->N; ++j) {
      if (j == self || o->kind[base + j] == TTRL_ABSENT) continue;
      if (o->lk && j < self) {  /* j acted before self: a changed target of j could abort self here */
        double d = lane_distance(o, R, base, self, j);
        if (-1.0 < d && d < desired_gap(o, P, base, self, j) + 1.0) link_at(o, base + self, j);
      }
      if (o->lane[base + j] != tgt && o->tgt[base + j] == tgt) {
        double d = lane_distance(o, R, base, self, j);
        double ds = desired_gap(o, P, base, self, j);
        mg(o, base + self, d, d);
        mg(o, base + self, d - ds, d);
        if (0 < d && d < ds) { o->tgt[base + self] = lane; break; }
      }
    }
    return;
  }
  mg(o, base + self, o->timer[base + self] - P->lane_change_delay, 0);
  if (!(P->lane_change_delay < o->timer[base + self])) return;   /* utils.do_every */
  o->timer[base + self] = 0;
  int cand[2], nc = 0;                                             /* RoadNetwork.side_lanes road.py:200-211 */
  if (R->lane_id[lane] > 0) cand[nc++] = lane - 1;
  if (R->lane_id[lane] < R->road_n[R->road[lane]] - 1) cand[nc++] = lane + 1;
  for (int k = 0; k < nc; ++k) {
    if (o->mg) {
      double s, r; local(R, cand[k], o->x[base + self], o->y[base + self], &s, &r);
      mg(o, base + self, 2 * R->width[cand[k]] - fabs(r), r);
      mg(o, base + self, s, s);
      mg(o, base + self, R->length[cand[k]] + P->lane_vehicle_length - s, s);
      mg(o, base + self, fabs(o->v[base + self]) - 1, 0);
    }
    if (!reachable(R, P, cand[k], o->x[base + self], o->y[base + self])) continue;
    if (fabs(o->v[base + self]) < 1) continue;
    if (mobil(o, R, P, base, self, cand[k])) o->tgt[base + self] = cand[k];
  }
}

/* ControlledVehicle.steering_control controller.py:145-187 */
static double steering_control(const S* o, const ttrl_lane_table_t* R, const ttrl_params_t* P, int base, int i, int l) {
  double s, r; local(R, l, o->x[base + i], o->y[base + i], &s, &r);
  double v = o->v[base + i];
  double lane_future_heading = heading_at(R, l, s + v * P->tau_pursuit);
  double lat_cmd = -P->kp_lateral * r;
  double hcmd = asin(clipd(lat_cmd / not_zero(v), -1, 1));
  double href = lane_future_heading + clipd(hcmd, -PI / 4, PI / 4);
  double hrate = P->kp_heading * wrap_to_pi(href - o->h[base + i]);
  double slip = asin(clipd(P->length / 2 / not_zero(v) * hrate, -1, 1));
  double st = atan(2 * tan(slip));
  return clipd(st, -P->max_steering, P->max_steering);
}

/* IDMVehicle.act behavior.py:93-137 */
static void idm_act(S* o, const ttrl_lane_table_t* R, const ttrl_params_t* P, int base, int i) {
  if (o->crashed[base + i]) return;
  follow_road(o, R, P, base, i);
  if (o->lc[base + i]) change_lane_policy(o, R, P, base, i);
  double st = steering_control(o, R, P, base, i, o->tgt[base + i]);
  st = clipd(st, -P->max_steering, P->max_steering);
  int f, r; neighbour(o, R, P, base, i, o->lane[base + i], &f, &r);
  double d = o->delta[base + i];
  double a = idm_acc(o, R, P, base, d, i, f);
  if (o->lane[base + i] != o->tgt[base + i]) {
    neighbour(o, R, P, base, i, o->tgt[base + i], &f, &r);
    double a2 = idm_acc(o, R, P, base, d, i, f);
    if (a2 < a) a = a2;                                        /* Python min(a, a2) */
  }
  o->acc[base + i] = clipd(a, -P->acc_max, P->acc_max);
  o->steer[base + i] = st;
}

/* ControlledVehicle.act controller.py:89-133 with action in {None, LANE_LEFT, LANE_RIGHT, IDLE} */
static void controlled_act(S* o, const ttrl_lane_table_t* R, const ttrl_params_t* P, int base, int i, int action) {
  follow_road(o, R, P, base, i);
  if (action == TTRL_LANE_RIGHT || action == TTRL_LANE_LEFT) {
    const int t = o->tgt[base + i], rd = R->road[t];
    int id = R->lane_id[t] + (action == TTRL_LANE_RIGHT ? 1 : -1);
    if (id < 0) id = 0;
    if (id > R->road_n[rd] - 1) id = R->road_n[rd] - 1;
    id += R->road_first[rd];
    if (reachable(R, P, id, o->x[base + i], o->y[base + i])) o->tgt[base + i] = id;
  }
  double st = steering_control(o, R, P, base, i, o->tgt[base + i]);
  double a = P->kp_a * (o->ts[base + i] - o->v[base + i]);
  o->steer[base + i] = clipd(st, -P->max_steering, P->max_steering);
  o->acc[base + i] = a;
}

/* MDPVehicle.speed_to_index controller.py:326-344 (np.round = half-to-even) */
static int speed_to_index(const ttrl_params_t* P, double v) {
  int n = P->n_target_speeds;
  double x = (v - P->target_speeds[0]) / (P->target_speeds[n - 1] - P->target_speeds[0]);
  return (int)clipd(nearbyint(x * (n - 1)), 0, n - 1);
}

/* MDPVehicle.act controller.py:295-315 */
static void mdp_act(S* o, const ttrl_lane_table_t* R, const ttrl_params_t* P, int base, int i, int action) {
  if (action == TTRL_FASTER || action == TTRL_SLOWER) {
    if (o->mg) {                                               /* np.round half-way point */
      const int n = P->n_target_speeds;
      const double x = (o->v[base + i] - P->target_speeds[0]) / (P->target_speeds[n - 1] - P->target_speeds[0]) * (n - 1);
      mg(o, base + i, x - floor(x) - 0.5, x);
    }
    int si = speed_to_index(P, o->v[base + i]) + (action == TTRL_FASTER ? 1 : -1);
    if (si < 0) si = 0;
    if (si > P->n_target_speeds - 1) si = P->n_target_speeds - 1;
    o->sidx[base + i] = si;
    o->ts[base + i] = P->target_speeds[si];
    controlled_act(o, R, P, base, i, -1);
    return;
  }
  controlled_act(o, R, P, base, i, action);
}

/* Vehicle.step kinematics.py:130-153 (+ clip_actions :155-168, on_state_update :170-177) */
static void vehicle_step(S* o, const ttrl_lane_table_t* R, const ttrl_params_t* P, int base, int i, double dt) {
  int k = base + i;
  if (o->kind[k] == TTRL_IDM) o->timer[k] += dt;                   /* IDMVehicle.step behavior.py:147 */
  if (o->crashed[k]) { o->steer[k] = 0; o->acc[k] = -1.0 * o->v[k]; }
  if (o->v[k] > P->max_speed) { double c = 1.0 * (P->max_speed - o->v[k]); if (c < o->acc[k]) o->acc[k] = c; }
  else if (o->v[k] < P->min_speed) { double c = 1.0 * (P->min_speed - o->v[k]); if (c > o->acc[k]) o->acc[k] = c; }
  double beta = atan(1.0 / 2 * tan(o->steer[k]));
  double vx = o->v[k] * cos(o->h[k] + beta), vy = o->v[k] * sin(o->h[k] + beta);
  o->x[k] += vx * dt; o->y[k] += vy * dt;
  if (o->hasimp[k]) { o->x[k] += o->ix[k]; o->y[k] += o->iy[k]; o->crashed[k] = 1; o->hasimp[k] = 0; }
  o->h[k] += o->v[k] * sin(beta) / (P->length / 2) * dt;
  o->v[k] += o->acc[k] * dt;
  o->lane[k] = closest_lane(R, o->x[k], o->y[k], o->h[k]);
  if (o->mg && R->n_lanes > 1) {                              /* argmin runner-up gap */
    double d1 = INFINITY, d2 = INFINITY;
    for (int l = 0; l < R->n_lanes; ++l) {
      double s, r; local(R, l, o->x[k], o->y[k], &s, &r);
      double ang = fabs(wrap_to_pi(o->h[k] - heading_at(R, l, s)));
      double a = s - R->length[l]; if (!(a > 0)) a = 0;
      double b = 0 - s; if (!(b > 0)) b = 0;
      double d = fabs(r) + a + b + 1.0 * ang;
      if (d < d1) { d2 = d1; d1 = d; } else if (d < d2) d2 = d;
    }
    mg(o, k, d2 - d1, d1);
  }
}

/* RoadObject.polygon objects.py:168-180 (closed: 5 points) */
static void polygon(const ttrl_params_t* P, double px, double py, double h, double pts[5][2]) {
  const double L = P->length, W = P->width;
  double c = cos(h), s = sin(h);
  double lx[4] = {-L / 2, -L / 2, +L / 2, +L / 2}, ly[4] = {-W / 2, +W / 2, +W / 2, -W / 2};
  for (int k = 0; k < 4; ++k) {
    pts[k][0] = c * lx[k] + (-s) * ly[k] + px;
    pts[k][1] = s * lx[k] + c * ly[k] + py;
  }
  pts[4][0] = pts[0][0]; pts[4][1] = pts[0][1];
}
static void project(double pts[5][2], double nx, double ny, double* mn, double* mx) {
  for (int k = 0; k < 5; ++k) {
    double p = pts[k][0] * nx + pts[k][1] * ny;
    if (k == 0 || p < *mn) *mn = p;
    if (k == 0 || p > *mx) *mx = p;
  }
}
static double interval_distance(double mina, double maxa, double minb, double maxb) {
  return mina < minb ? minb - maxa : mina - maxb;                /* utils.py:186-191 */
}
/* utils.are_polygons_intersecting utils.py:194-239 */
static void sat(double a[5][2], double b[5][2], double dax, double day, double dbx, double dby,
                int* inter, int* will, double* tx, double* ty, double* smg, int* smg_line) {
  int it = 1, wi = 1; double mind = INFINITY, axx = 0, axy = 0;
  double (*polys[2])[2] = {a, b};
  double cand_d[8], cand_x[8], cand_y[8]; int nc = 0;            /* margins: every axis's |dist|, axis */
  for (int pi = 0; pi < 2; ++pi) {
    double (*pg)[2] = polys[pi];
    for (int e = 0; e < 4; ++e) {
      double nx = -pg[e + 1][1] + pg[e][1], ny = pg[e + 1][0] - pg[e][0];
      double nn = sqrt(nx * nx + ny * ny);
      nx /= nn; ny /= nn;
      double mina = 0, maxa = 0, minb = 0, maxb = 0;
      project(a, nx, ny, &mina, &maxa);
      project(b, nx, ny, &minb, &maxb);
      const double scale = fabs(mina) + fabs(maxb);
      if (smg) {  /* the separation test, and the branch of interval_distance where its two values differ */
        double m0 = fabs(interval_distance(mina, maxa, minb, maxb)) / (1 + scale);
        if (m0 < *smg) { *smg = m0; *smg_line = __LINE__; }
        if (fabs((minb - maxa) - (mina - maxb)) > 1e-9 * (1 + scale)) {
          double m1 = fabs(mina - minb) / (1 + scale);
          if (m1 < *smg) { *smg = m1; *smg_line = __LINE__; }
        }
      }
      if (interval_distance(mina, maxa, minb, maxb) > 0) it = 0;
      double vp = nx * (dax - dbx) + ny * (day - dby);
      if (vp < 0) mina += vp; else maxa += vp;
      double dist = interval_distance(mina, maxa, minb, maxb);
      if (smg) {
        double m2 = fabs(dist) / (1 + scale);
        if (m2 < *smg) { *smg = m2; *smg_line = __LINE__; }
        if (fabs((minb - maxa) - (mina - maxb)) > 1e-9 * (1 + scale)) {
          double m3 = fabs(mina - minb) / (1 + scale);
          if (m3 < *smg) { *smg = m3; *smg_line = __LINE__; }
        }
      }
      if (dist > 0) wi = 0;
      if (!it && !wi) break;
      double cax = (((a[0][0] + a[1][0]) + a[2][0]) + a[3][0]) / 4, cay = (((a[0][1] + a[1][1]) + a[2][1]) + a[3][1]) / 4;
      double cbx = (((b[0][0] + b[1][0]) + b[2][0]) + b[3][0]) / 4, cby = (((b[0][1] + b[1][1]) + b[2][1]) + b[3][1]) / 4;
      double dx = cax - cbx, dy = cay - cby;
      const double sgnd = dx * nx + dy * ny;
      if (smg) {
        cand_d[nc] = fabs(dist); cand_x[nc] = sgnd > 0 ? nx : -nx; cand_y[nc] = sgnd > 0 ? ny : -ny; ++nc;
        const double m4 = fabs(sgnd) / (1 + fabs(dx) + fabs(dy));  /* the translation's sign choice */
        if (fabs(dist) > 1e-9 && m4 < *smg) { *smg = m4; *smg_line = __LINE__; }
      }
      if (fabs(dist) < mind) {
        mind = fabs(dist);
        if (sgnd > 0) { axx = nx; axy = ny; } else { axx = -nx; axy = -ny; }
      }
    }
  }
  *inter = it; *will = wi;
  *tx = wi ? mind * axx : 0; *ty = wi ? mind * axy : 0;
  if (smg && wi) {  /* the translation: argmin of |dist| over the axes whose translation differs */
    for (int q = 0; q < nc; ++q) {
      const double jump = fabs(cand_d[q] * cand_x[q] - mind * axx) + fabs(cand_d[q] * cand_y[q] - mind * axy);
      if (jump <= 1e-9) continue;                                  /* the winner, or the same push */
      const double m = (cand_d[q] - mind) / (1 + mind);
      if (m < *smg) { *smg = m; *smg_line = __LINE__; }
    }
  }
}

/* RoadObject.handle_collisions objects.py:91-137 for a vehicle pair i<j */
static void handle_collisions(S* o, const ttrl_params_t* P, int base, int i, int j, double dt) {
  int a = base + i, b = base + j;
  double dx = o->x[b] - o->x[a], dy = o->y[b] - o->y[a];
  const double thr = (P->diagonal + P->diagonal) / 2 + o->v[a] * dt;
  if (o->mg) {
    mg(o, a, sqrt(dx * dx + dy * dy) - thr, o->x[a]);
    mg(o, b, sqrt(dx * dx + dy * dy) - thr, o->x[a]);
  }
  if (o->lk && sqrt(dx * dx + dy * dy) <= thr + 1.0) {  /* a pair the prefilter may pass: each reads the other */
    link_at(o, a, j);
    link_at(o, b, i);
  }
  if (sqrt(dx * dx + dy * dy) > thr) return;
  double pa[5][2], pb[5][2];
  polygon(P, o->x[a], o->y[a], o->h[a], pa);
  polygon(P, o->x[b], o->y[b], o->h[b], pb);
  double ca = cos(o->h[a]), sa = sin(o->h[a]), cb = cos(o->h[b]), sb = sin(o->h[b]);
  double dax = o->v[a] * ca * dt, day = o->v[a] * sa * dt, dbx = o->v[b] * cb * dt, dby = o->v[b] * sb * dt;
  int inter, will; double tx, ty;
  double smg = INFINITY; int smg_line = 0;
  sat(pa, pb, dax, day, dbx, dby, &inter, &will, &tx, &ty, o->mg ? &smg : NULL, &smg_line);
  if (o->mg && smg < INFINITY) { mg_at(o, a, smg, 0, smg_line); mg_at(o, b, smg, 0, smg_line); }
  if (will) {
    o->ix[a] = tx / 2; o->iy[a] = ty / 2; o->hasimp[a] = 1;
    o->ix[b] = -tx / 2; o->iy[b] = -ty / 2; o->hasimp[b] = 1;
  }
  if (inter) { o->crashed[a] = 1; o->crashed[b] = 1; }
}

/* ---------------------------------------------------------------- RegulatedRoad (regulation.py) */
/* RoadNetwork.position_heading_along_route road.py:352-389 for ControlledVehicle.
 * predict_trajectory_constant_speed controller.py:228-247 at times 0.25 .. 2.75 (np.arange(0.25, 3, 0.25)) */
enum { PRED_T = 11 };
static void predict(const S* o, const ttrl_lane_table_t* R, int k, double px[PRED_T], double py[PRED_T],
                    double ph[PRED_T]) {
  const int cur = o->lane[k];
  double s0, r0; local(R, cur, o->x[k], o->y[k], &s0, &r0);
  const int n = (o->rn && o->rn[k] > 0) ? o->rn[k] : 1;     /* route or [lane_index] */
  const int8_t* rr = o->rn ? o->rroad + (size_t)k * TTRL_ROUTE_MAX : 0;
  const int8_t* rl = o->rn ? o->rlane + (size_t)k * TTRL_ROUTE_MAX : 0;
  const int use_route = o->rn && o->rn[k] > 0;
  for (int t = 0; t < PRED_T; ++t) {
    const double tt = 0.25 + t * 0.25;
    double L = s0 + o->v[k] * tt;
    int idx = 0, lane;
#define RESOLVE(q) (use_route ? R->road_first[rr[q]] + (rl[q] >= 0 ? rl[q] \
                      : (R->lane_id[cur] < R->road_n[R->road[cur]] ? R->lane_id[cur] : 0)) : cur)
    lane = RESOLVE(0);
    while (n - idx > 1 && L > R->length[lane]) { L -= R->length[lane]; ++idx; lane = RESOLVE(idx); }
#undef RESOLVE
    position(R, lane, L, 0, &px[t], &py[t]);
    ph[t] = heading_at(R, lane, L);
  }
}
/* utils.point_in_rotated_rectangle utils.py:75-91 (rotation by +angle, as written) */
static int point_in_rect(double x, double y, double cx, double cy, double l, double w, double a) {
  double c = cos(a), s = sin(a);
  double dx = x - cx, dy = y - cy;
  double u = c * dx + (-s) * dy, v = s * dx + c * dy;
  return -l / 2 <= u && u <= l / 2 && -w / 2 <= v && v <= w / 2;
}
/* utils.has_corner_inside utils.py:158-172 over rect_corners(include_midpoints, include_center) :126-155 */
static int corner_inside(double c1x, double c1y, double l1, double w1, double a1, double c2x, double c2y, double l2,
                         double w2, double a2) {
  const double hl = l1 / 2, hw = w1 / 2;
  const double px[9] = {-hl, -hl, hl, hl, 0, -hl, hl, 0, 0};
  const double py[9] = {-hw, hw, hw, -hw, 0, 0, 0, -hw, hw};
  double c = cos(a1), s = sin(a1);
  for (int q = 0; q < 9; ++q) {
    double x = c * px[q] + (-s) * py[q] + c1x, y = s * px[q] + c * py[q] + c1y;
    if (point_in_rect(x, y, c2x, c2y, l2, w2, a2)) return 1;
  }
  return 0;
}
/* RegulatedRoad.is_conflict_possible regulation.py:80-103 */
static int conflict(const ttrl_params_t* P, const double* ax, const double* ay, const double* ah, const double* bx,
                    const double* by, const double* bh) {
  const double l = 1.5 * P->length, w = 0.9 * P->width;
  for (int t = 0; t < PRED_T; ++t) {
    double dx = bx[t] - ax[t], dy = by[t] - ay[t];
    if (sqrt(dx * dx + dy * dy) > P->length) continue;
    if (corner_inside(ax[t], ay[t], l, w, ah[t], bx[t], by[t], l, w, bh[t]) ||
        corner_inside(bx[t], by[t], l, w, bh[t], ax[t], ay[t], l, w, ah[t]))
      return 1;
  }
  return 0;
}
/* The signed decision value of conflict() (>= 0 iff a conflict): per time step, min(LENGTH - the
 * centre distance, the larger corner-inside value of the two rectangles), where a rectangle's
 * corner-inside value is the max over its 9 points of min(l/2 - |u|, w/2 - |v|) in the other's
 * frame -- its magnitude is the margin of the float64 decision (oracle_frame_margins only). */
static double inside_value(double c1x, double c1y, double l1, double w1, double a1, double c2x, double c2y, double l2,
                           double w2, double a2) {
  const double hl = l1 / 2, hw = w1 / 2;
  const double px[9] = {-hl, -hl, hl, hl, 0, -hl, hl, 0, 0};
  const double py[9] = {-hw, hw, hw, -hw, 0, 0, 0, -hw, hw};
  double c = cos(a1), s = sin(a1), best = -INFINITY;
  for (int q = 0; q < 9; ++q) {
    double x = c * px[q] + (-s) * py[q] + c1x, y = s * px[q] + c * py[q] + c1y;
    double c2 = cos(a2), s2 = sin(a2), dx = x - c2x, dy = y - c2y;
    double u = c2 * dx + (-s2) * dy, v = s2 * dx + c2 * dy;
    double du = l2 / 2 - fabs(u), dv = w2 / 2 - fabs(v);
    double m = du < dv ? du : dv;
    if (m > best) best = m;
  }
  return best;
}
static double conflict_value(const ttrl_params_t* P, const double* ax, const double* ay, const double* ah,
                             const double* bx, const double* by, const double* bh) {
  const double l = 1.5 * P->length, w = 0.9 * P->width;
  double best = -INFINITY;
  for (int t = 0; t < PRED_T; ++t) {
    double dx = bx[t] - ax[t], dy = by[t] - ay[t];
    double g = P->length - sqrt(dx * dx + dy * dy);
    double ci = inside_value(ax[t], ay[t], l, w, ah[t], bx[t], by[t], l, w, bh[t]);
    double cj = inside_value(bx[t], by[t], l, w, bh[t], ax[t], ay[t], l, w, ah[t]);
    double c = ci > cj ? ci : cj;
    if (c < g) g = c;
    if (g > best) best = g;
  }
  return best;
}

/* RegulatedRoad.respect_priorities regulation.py:62-77 (front_distance_to objects.py:204-205) */
static int respect(const S* o, const ttrl_lane_table_t* R, int a, int b) {
  const int pa = R->priority[o->lane[a]], pb = R->priority[o->lane[b]];
  if (pa > pb) return b;
  if (pa < pb) return a;
  double fab = cos(o->h[a]) * (o->x[b] - o->x[a]) + sin(o->h[a]) * (o->y[b] - o->y[a]);
  double fba = cos(o->h[b]) * (o->x[a] - o->x[b]) + sin(o->h[b]) * (o->y[a] - o->y[b]);
  return fab > fba ? a : b;
}
/* RegulatedRoad.enforce_road_rules regulation.py:34-60 (YIELD_DURATION = 0: a yield lasts until
 * the next enforcement) */
static void enforce_road_rules(S* o, const ttrl_lane_table_t* R, const ttrl_params_t* P, int base) {
  const int N = o->N;
  for (int i = 0; i < N; ++i) {
    const int k = base + i;
    if (o->kind[k] != TTRL_ABSENT && o->yield[k]) { o->ts[k] = R->speed_limit[o->lane[k]]; o->yield[k] = 0; }
  }
  double* px = malloc(sizeof(double) * 3 * PRED_T * N);
  double *py = px + PRED_T * N, *ph = py + PRED_T * N;
  for (int i = 0; i < N; ++i)
    if (o->kind[base + i] != TTRL_ABSENT) predict(o, R, base + i, px + PRED_T * i, py + PRED_T * i, ph + PRED_T * i);
  for (int i = 0; i < N; ++i) {
    if (o->kind[base + i] == TTRL_ABSENT) continue;
    for (int j = i + 1; j < N; ++j) {
      if (o->kind[base + j] == TTRL_ABSENT) continue;
      if (o->mg) {  /* the conflict test and the front-distance comparison decide for both vehicles */
        const double cv = conflict_value(P, px + PRED_T * i, py + PRED_T * i, ph + PRED_T * i, px + PRED_T * j,
                                         py + PRED_T * j, ph + PRED_T * j);
        const double sc = fabs(o->x[base + i]) + fabs(o->y[base + i]);
        mg(o, base + i, cv, sc);
        mg(o, base + j, cv, sc);
        const int a = base + i, b = base + j;
        if (cv >= 0 && R->priority[o->lane[a]] == R->priority[o->lane[b]]) {  /* respect() runs */
          double fab = cos(o->h[a]) * (o->x[b] - o->x[a]) + sin(o->h[a]) * (o->y[b] - o->y[a]);
          double fba = cos(o->h[b]) * (o->x[a] - o->x[b]) + sin(o->h[b]) * (o->y[a] - o->y[b]);
          mg(o, a, fab - fba, sc);
          mg(o, b, fab - fba, sc);
        }
      }
      if (!conflict(P, px + PRED_T * i, py + PRED_T * i, ph + PRED_T * i, px + PRED_T * j, py + PRED_T * j,
                    ph + PRED_T * j))
        continue;
      const int y = respect(o, R, base + i, base + j);
      if (o->kind[y] == TTRL_IDM) { o->ts[y] = 0; o->yield[y] = 1; }
    }
  }
  free(px);
}

static int check(const ttrl_state_t* s) {
  if (!s || s->dtype != TTRL_F64 || s->n_envs < 0 || s->n_veh <= 0) return TTRL_E_ARG;
  return 0;
}

int oracle_meta_action(const ttrl_state_t* s, const ttrl_lane_table_t* R, const ttrl_params_t* P,
                       const int32_t* actions, void* stream) {
  (void)stream; if (check(s)) return TTRL_E_ARG;
  S o = view(s);
  for (int e = 0; e < o.E; ++e)
    if (actions[e] < 0 || actions[e] > 4) return TTRL_E_ARG;
  for (int e = 0; e < o.E; ++e) {
    int base = e * o.N;
    for (int i = 0; i < o.N; ++i)             /* the env's controlled vehicle: its first MDPVehicle */
      if (o.kind[base + i] == TTRL_MDP) { mdp_act(&o, R, P, base, i, actions[e]); break; }
  }
  return 0;
}

/* Road.act road.py:461-464, one env */
static void act_env(S* o, const ttrl_lane_table_t* R, const ttrl_params_t* P, int e) {
  int base = e * o->N;
  for (int i = 0; i < o->N; ++i) {
    if (o->kind[base + i] == TTRL_MDP) controlled_act(o, R, P, base, i, -1);
    else if (o->kind[base + i] == TTRL_IDM) idm_act(o, R, P, base, i);
  }
}

/* Road.step road.py:466-478, one env */
static void step_env(S* o, const ttrl_lane_table_t* R, const ttrl_params_t* P, int e, double dt) {
  int base = e * o->N;
  if (R->regulation_frequency > 0 && o->reg) {               /* RegulatedRoad.step regulation.py:28-32 */
    o->reg[e] += 1;
    const int period = (int)(1.0 / dt / R->regulation_frequency);
    if (period > 0 && o->reg[e] % period == 0) enforce_road_rules(o, R, P, base);
  }
  for (int i = 0; i < o->N; ++i)
    if (o->kind[base + i] != TTRL_ABSENT) vehicle_step(o, R, P, base, i, dt);
  for (int i = 0; i < o->N; ++i) {
    if (o->kind[base + i] == TTRL_ABSENT) continue;
    for (int j = i + 1; j < o->N; ++j)
      if (o->kind[base + j] != TTRL_ABSENT) handle_collisions(o, P, base, i, j, dt);
  }
}

int oracle_road_act(const ttrl_state_t* s, const ttrl_lane_table_t* R, const ttrl_params_t* P, void* stream) {
  (void)stream; if (check(s)) return TTRL_E_ARG;
  S o = view(s);
#pragma omp parallel for schedule(static)
  for (int e = 0; e < o.E; ++e) act_env(&o, R, P, e);
  return 0;
}

int oracle_road_step(const ttrl_state_t* s, const ttrl_lane_table_t* R, const ttrl_params_t* P, double dt, void* stream) {
  (void)stream; if (check(s)) return TTRL_E_ARG;
  S o = view(s);
#pragma omp parallel for schedule(static)
  for (int e = 0; e < o.E; ++e) step_env(&o, R, P, e, dt);
  return 0;
}

/* AbstractEnv._simulate abstract.py:252-282 */
int oracle_simulate(const ttrl_state_t* s, const ttrl_lane_table_t* R, const ttrl_params_t* P,
                    const int32_t* actions, int32_t frames, double dt, void* stream) {
  if (check(s)) return TTRL_E_ARG;
  for (int f = 0; f < frames; ++f) {
    int rc;
    if (f == 0 && actions && (rc = oracle_meta_action(s, R, P, actions, stream))) return rc;
    if ((rc = oracle_road_act(s, R, P, stream))) return rc;
    if ((rc = oracle_road_step(s, R, P, dt, stream))) return rc;
  }
  return 0;
}

/* One frame (the meta-action first when `actions` is given, then Road.act if phases & 1 and
 * Road.step(dt) if phases & 2) with every discrete decision's float64 margin recorded per vehicle
 * into margin[E*N] (see mg()) and its source line into site[E*N]: the classifier of float32
 * decision flips (SURVEY.md §8(d) parity tolerance). */
int oracle_frame_links(const ttrl_state_t* s, const ttrl_lane_table_t* R, const ttrl_params_t* P,
                       const int32_t* actions, double dt, int32_t phases, double* margin, int32_t* site,
                       int32_t* links, int32_t link_max) {
  if (check(s) || !margin || (links && link_max < 1)) return TTRL_E_ARG;
  S o = view(s);
  for (int k = 0; k < o.E * o.N; ++k) { margin[k] = INFINITY; if (site) site[k] = 0; }
  o.mg = margin; o.mgsite = site;
  if (links) {
    for (size_t q = 0; q < (size_t)o.E * o.N * link_max; ++q) links[q] = -1;
    o.lk = links; o.lkmax = link_max;
  }
  for (int e = 0; e < o.E; ++e)
    if (actions && (actions[e] < 0 || actions[e] > 4)) return TTRL_E_ARG;
#pragma omp parallel for schedule(static)
  for (int e = 0; e < o.E; ++e) {
    const int base = e * o.N;
    if (actions)
      for (int i = 0; i < o.N; ++i)
        if (o.kind[base + i] == TTRL_MDP) { mdp_act(&o, R, P, base, i, actions[e]); break; }
    if (phases & 1) act_env(&o, R, P, e);
    if (phases & 2) step_env(&o, R, P, e, dt);
  }
  return 0;
}

int oracle_frame_margins(const ttrl_state_t* s, const ttrl_lane_table_t* R, const ttrl_params_t* P,
                         const int32_t* actions, double dt, int32_t phases, double* margin, int32_t* site) {
  return oracle_frame_links(s, R, P, actions, dt, phases, margin, site, NULL, 0);
}

int oracle_neighbours(const ttrl_state_t* s, const ttrl_lane_table_t* R, const ttrl_params_t* P,
                      const int32_t* query_lane, int32_t* front, int32_t* rear) {
  if (check(s)) return TTRL_E_ARG;
  S o = view(s);
  for (int e = 0; e < o.E; ++e)
    for (int i = 0; i < o.N; ++i) {
      int k = e * o.N + i, f = -1, r = -1;
      if (o.kind[k] != TTRL_ABSENT) {
        int l = query_lane && query_lane[k] >= 0 ? query_lane[k] : o.lane[k];
        neighbour(&o, R, P, e * o.N, i, l, &f, &r);
      }
      front[k] = f; rear[k] = r;
    }
  return 0;
}

/* AbstractEnv.vehicle: the env's controlled vehicle, its first MDPVehicle in list order
 * (slot 0 on the highway; appended after the traffic in IntersectionEnv._make_vehicles). */
static int ego_of(const S* o, int base) {
  for (int i = 0; i < o->N; ++i)
    if (o->kind[base + i] == TTRL_MDP) return i;
  return -1;
}

/* ---------------------------------------------------------------- observations */
/* Vehicle.to_dict kinematics.py:237-261 (route None => cos_d = sin_d = 0) */
static double feature(const S* o, const ttrl_lane_table_t* R, int k, int f) {
  double c = cos(o->h[k]), sn = sin(o->h[k]);
  switch (f) {
    case TTRL_F_PRESENCE: return 1;
    case TTRL_F_X: return o->x[k];
    case TTRL_F_Y: return o->y[k];
    case TTRL_F_VX: return o->v[k] * c;
    case TTRL_F_VY: return o->v[k] * sn;
    case TTRL_F_HEADING: return o->h[k];
    case TTRL_F_COS_H: return c;
    case TTRL_F_SIN_H: return sn;
    case TTRL_F_COS_D: case TTRL_F_SIN_D: return 0;
    case TTRL_F_LONG_OFF: case TTRL_F_LAT_OFF: case TTRL_F_ANG_OFF: {
      double s, r; local(R, o->lane[k], o->x[k], o->y[k], &s, &r);
      if (f == TTRL_F_LONG_OFF) return s;
      if (f == TTRL_F_LAT_OFF) return r;
      return wrap_to_pi(o->h[k] - heading_at(R, o->lane[k], s));  /* local_angle lane.py:145-147 */
    }
  }
  return 0;
}

/* KinematicObservation.observe observation.py:233-275: order sorted, shuffled with the env's
 * np_random (order_shuffled 2: np_random.shuffle(obs[1:]), :272-273), or ids only (1). */
int oracle_observe_kinematics(const ttrl_state_t* s, const ttrl_lane_table_t* R, const ttrl_params_t* P,
                              const ttrl_kin_cfg_t* cfg, const uint8_t* mask, float* out, int32_t* ids) {
  if (check(s)) return TTRL_E_ARG;
  if (cfg->order_shuffled == 2 && (!s->rng || cfg->vehicles_count - 1 > 64)) return TTRL_E_ARG;
  S o = view(s);
  const int V = cfg->vehicles_count, F = cfg->n_features;
#pragma omp parallel
  {
  int* cand = (int*)malloc(sizeof(int) * o.N);
  double* key = (double*)malloc(sizeof(double) * o.N);
#pragma omp for schedule(static)
  for (int e = 0; e < o.E; ++e) {
    if (mask && !mask[e]) continue;
    int base = e * o.N, ei = ego_of(&o, base), ego = base + (ei < 0 ? 0 : ei);
    float* ob = out + (size_t)e * V * F;
    int nc = 0;
    for (int j = 0; j < o.N && ei >= 0; ++j) {   /* Road.close_objects_to road.py:427-433 */
      int k = base + j;
      if (j == ei || o.kind[k] == TTRL_ABSENT) continue;
      double dx = o.x[k] - o.x[ego], dy = o.y[k] - o.y[ego];
      if (!(sqrt(dx * dx + dy * dy) < cfg->perception_distance)) continue;
      double ld = lane_distance(&o, R, base, ei, j);
      if (!cfg->see_behind && !(-2 * P->length < ld)) continue;
      cand[nc] = j; key[nc] = fabs(ld); nc++;
    }
    /* stable insertion sort by |lane distance| (sorted(), road.py:444) */
    if (!cfg->order_shuffled)
      for (int a = 1; a < nc; ++a) {
        int cj = cand[a]; double ck = key[a]; int b = a - 1;
        while (b >= 0 && key[b] > ck) { cand[b + 1] = cand[b]; key[b + 1] = key[b]; b--; }
        cand[b + 1] = cj; key[b + 1] = ck;
      }
    if (nc > V - 1) nc = V - 1;
    int perm[64];                                 /* output row 1 + t holds candidate row perm[t] */
    for (int t = 0; t < V - 1 && t < 64; ++t) perm[t] = t;
    if (cfg->order_shuffled == 2 && V - 1 > 1) {  /* Generator.shuffle: random_interval swaps */
      pcg_t g; rng_load(&g, o.rng + (size_t)e * TTRL_RNG_WORDS);
      for (int i = V - 2; i >= 1; --i) {
        const int j = (int)pcg_interval(&g, (uint64_t)i);
        const int t = perm[i]; perm[i] = perm[j]; perm[j] = t;
      }
      rng_store(&g, o.rng + (size_t)e * TTRL_RNG_WORDS);
    }
    for (int r = 0; r < V; ++r) {
      const int q = r == 0 ? -1 : (cfg->order_shuffled == 2 ? perm[r - 1] : r - 1);
      for (int c = 0; c < F; ++c) {
        double val = 0;
        if (ei >= 0 && (r == 0 || q < nc)) {
          int k = r == 0 ? ego : base + cand[q];
          int f = cfg->features[c];
          val = feature(&o, R, k, f);
          if (r > 0 && !cfg->absolute && (f == TTRL_F_X || f == TTRL_F_Y || f == TTRL_F_VX || f == TTRL_F_VY))
            val -= feature(&o, R, ego, f);
          if (cfg->normalize && cfg->has_range[f]) {
            val = lmap(val, cfg->range_lo[f], cfg->range_hi[f], -1, 1);
            if (cfg->clip) val = clipd(val, -1, 1);
          }
        }
        ob[r * F + c] = (float)val;
      }
    }
    if (ids)
      for (int r = 0; r < V - 1; ++r) ids[e * (V - 1) + r] = r < nc ? cand[r] : -1;
  }
  free(cand); free(key);
  }
  return 0;
}

/* Observation decision margins (the float32 observation classifier, tests/test_gpu_parity.py):
 * every output cell records the smallest relative margin of a discrete decision that could move
 * content into or out of it (a floor() cell index, a range test, a min comparison); +inf where
 * none.  Like mg(), a float32 observer may differ from the float64 one in a cell only where this
 * margin is below the float32 working precision. */
static void mg_cell(double* m, size_t q, double v) { if (m && v < m[q]) m[q] = v; }

/* The cell (floor(ux), floor(uy)) of a layer [W][H], its neighbour across the nearer boundary of
 * each axis, and the diagonal one: the cells a small error in (ux, uy) can move an item between.
 * Margins in metres (distance to the boundary) relative to `scale`. */
static void grid_item_mg(double* m, int W, int H, double ux, double uy, double sx, double sy, double scale) {
  const double cx = floor(ux), cy = floor(uy), fx = ux - cx, fy = uy - cy;
  const double mx = (fx < 0.5 ? fx : 1 - fx) * sx / scale, my = (fy < 0.5 ? fy : 1 - fy) * sy / scale;
  const int dx = fx < 0.5 ? -1 : 1, dy = fy < 0.5 ? -1 : 1;
  const double cand[4][3] = {{cx, cy, mx < my ? mx : my}, {cx + dx, cy, mx}, {cx, cy + dy, my},
                             {cx + dx, cy + dy, mx > my ? mx : my}};
  for (int q = 0; q < 4; ++q)
    if (0 <= cand[q][0] && cand[q][0] < W && 0 <= cand[q][1] && cand[q][1] < H)
      mg_cell(m, (size_t)cand[q][0] * H + (size_t)cand[q][1], cand[q][2]);
}

/* OccupancyGridObservation.observe observation.py:353-434 (+ fill_road_layer_by_lanes :453-483);
 * margin (optional, [E][F][W][H]): see grid_item_mg */
int oracle_observe_grid_m(const ttrl_state_t* s, const ttrl_lane_table_t* R, const ttrl_params_t* P,
                          const ttrl_grid_cfg_t* cfg, float* out, double* margin) {
  (void)P; if (check(s)) return TTRL_E_ARG;
  S o = view(s);
  const int F = cfg->n_features, W = cfg->shape_x, H = cfg->shape_y;
  if (margin)
    for (size_t q = 0; q < (size_t)o.E * F * W * H; ++q) margin[q] = INFINITY;
#pragma omp parallel
  {
  double* grid = (double*)malloc(sizeof(double) * F * W * H);
#pragma omp for schedule(static)
  for (int e = 0; e < o.E; ++e) {
    int base = e * o.N, ei = ego_of(&o, base), ego = base + ei;
    for (int q = 0; q < F * W * H; ++q) grid[q] = NAN;
    if (ei < 0) {
      for (int q = 0; q < F * W * H; ++q) out[(size_t)e * F * W * H + q] = 0.0f;
      continue;
    }
    for (int c = 0; c < F; ++c) {
      int f = cfg->features[c];
      if (f == TTRL_F_ON_ROAD) {
        double spacing = cfg->step_x < cfg->step_y ? cfg->step_x : cfg->step_y;
        for (int l = 0; l < R->n_lanes; ++l) {
          double origin, rr; local(R, l, o.x[ego], o.y[ego], &origin, &rr);
          double start = origin - cfg->lane_perception_distance, stop = origin + cfg->lane_perception_distance;
          long n = (long)ceil((stop - start) / spacing);           /* np.arange length */
          double d1 = (start + spacing) - start;                    /* numpy fill: delta = buf[1]-buf[0] */
          for (long i = 0; i < n; ++i) {
            double wp = i == 0 ? start : (i == 1 ? start + spacing : start + i * d1);
            wp = clipd(wp, 0, R->length[l]);
            double px, py;
            position(R, l, wp, 0, &px, &py);
            const double scale = 1 + fabs(px) + fabs(py);
            px -= o.x[ego]; py -= o.y[ego];
            long cx = (long)floor((px - cfg->grid_min_x) / cfg->step_x);
            long cy = (long)floor((py - cfg->grid_min_y) / cfg->step_y);
            if (0 <= cx && cx < W && 0 <= cy && cy < H) grid[(c * W + cx) * H + cy] = 1;
            if (margin)
              grid_item_mg(margin + ((size_t)e * F + c) * W * H, W, H, (px - cfg->grid_min_x) / cfg->step_x,
                           (py - cfg->grid_min_y) / cfg->step_y, cfg->step_x, cfg->step_y, scale);
          }
        }
        continue;
      }
      for (int j = o.N - 1; j >= 0; --j) {        /* df[::-1].iterrows(): lowest index wins */
        int k = base + j;
        if (o.kind[k] == TTRL_ABSENT) continue;
        double x = o.x[k] - o.x[ego], y = o.y[k] - o.y[ego];
        double val = feature(&o, R, k, f);
        if (f == TTRL_F_X || f == TTRL_F_Y || f == TTRL_F_VX || f == TTRL_F_VY) val -= feature(&o, R, ego, f);
        if (cfg->has_range[f]) val = lmap(val, cfg->range_lo[f], cfg->range_hi[f], -1, 1);
        if (cfg->has_range[TTRL_F_X]) {
          x = lmap(x, cfg->range_lo[TTRL_F_X], cfg->range_hi[TTRL_F_X], -1, 1);
          x = lmap(x, -1, 1, cfg->range_lo[TTRL_F_X], cfg->range_hi[TTRL_F_X]);
        }
        if (cfg->has_range[TTRL_F_Y]) {
          y = lmap(y, cfg->range_lo[TTRL_F_Y], cfg->range_hi[TTRL_F_Y], -1, 1);
          y = lmap(y, -1, 1, cfg->range_lo[TTRL_F_Y], cfg->range_hi[TTRL_F_Y]);
        }
        long cx = (long)floor((x - cfg->grid_min_x) / cfg->step_x);
        long cy = (long)floor((y - cfg->grid_min_y) / cfg->step_y);
        if (0 <= cx && cx < W && 0 <= cy && cy < H) grid[(c * W + cx) * H + cy] = val;
        if (margin)
          grid_item_mg(margin + ((size_t)e * F + c) * W * H, W, H, (x - cfg->grid_min_x) / cfg->step_x,
                       (y - cfg->grid_min_y) / cfg->step_y, cfg->step_x, cfg->step_y,
                       1 + fabs(o.x[k]) + fabs(o.y[k]) + fabs(o.x[ego]) + fabs(o.y[ego]));
      }
    }
    float* ob = out + (size_t)e * F * W * H;
    for (int q = 0; q < F * W * H; ++q) {
      double g = grid[q];
      if (cfg->clip && g == g) g = clipd(g, -1, 1);
      ob[q] = (float)(g == g ? g : 0.0);
    }
  }
  free(grid);
  }
  return 0;
}

int oracle_observe_grid(const ttrl_state_t* s, const ttrl_lane_table_t* R, const ttrl_params_t* P,
                        const ttrl_grid_cfg_t* cfg, float* out) {
  return oracle_observe_grid_m(s, R, P, cfg, out, NULL);
}

/* ---------------------------------------------------------------- scene generation */
/* highway scene, SURVEY.md §3.C: ego MDPVehicle then create_random + randomize_behavior */
int oracle_reset_highway(const ttrl_state_t* s, const ttrl_lane_table_t* R, const ttrl_params_t* P,
                         const ttrl_reset_cfg_t* cfg, const uint64_t* pcg) {
  if (check(s) || cfg->n_vehicles > s->n_veh || cfg->n_vehicles < 1) return TTRL_E_ARG;
  S o = view(s);
#pragma omp parallel for schedule(static)
  for (int e = 0; e < o.E; ++e) {
    int base = e * o.N;
    pcg_t g;
    g.st = ((unsigned __int128)pcg[4 * e] << 64) | pcg[4 * e + 1];
    g.inc = ((unsigned __int128)pcg[4 * e + 2] << 64) | pcg[4 * e + 3];
    g.has32 = 0; g.u32 = 0;
    for (int i = 0; i < o.N; ++i) {
      int k = base + i;
      o.kind[k] = TTRL_ABSENT; o.crashed[k] = 0; o.hasimp[k] = 0; o.lc[k] = 0;
      o.x[k] = o.y[k] = o.h[k] = o.v[k] = o.ts[k] = o.timer[k] = o.steer[k] = o.acc[k] = 0;
      o.ix[k] = o.iy[k] = 0; o.delta[k] = 4.0; o.lane[k] = o.tgt[k] = 0; o.sidx[k] = -1;
    }
    /* ego: MDPVehicle(road, lane.position(x, 0), lane.heading_at(x), speed) */
    int l = cfg->ego_lane;
    double ex, ey;
    position(R, l, cfg->ego_x, 0.0, &ex, &ey);
    const double eh = heading_at(R, l, cfg->ego_x);
    o.kind[base] = TTRL_MDP; o.x[base] = ex; o.y[base] = ey; o.h[base] = eh; o.v[base] = cfg->ego_speed;
    o.lane[base] = o.tgt[base] = closest_lane(R, ex, ey, eh);
    o.sidx[base] = speed_to_index(P, cfg->ego_speed);
    o.ts[base] = P->target_speeds[o.sidx[base]];
    for (int i = 1; i < cfg->n_vehicles; ++i) {
      int k = base + i;
      int lid = (int)pcg_bounded(&g, (uint32_t)R->n_lanes);          /* choice(len(lanes)) */
      double sp = pcg_uniform(&g, cfg->speed_lo, cfg->speed_hi);
      double offset = cfg->spacing * (12 + 1.0 * sp) * cfg->density_factor;
      double x0 = 0; int have = 0;
      for (int j = 0; j < i; ++j) {
        double sj, rj; local(R, lid, o.x[base + j], o.y[base + j], &sj, &rj);
        if (!have || sj > x0) { x0 = sj; have = 1; }
      }
      x0 += offset * pcg_uniform(&g, 0.9, 1.1);
      o.kind[k] = TTRL_IDM; o.lc[k] = (uint8_t)cfg->lane_change;
      position(R, lid, x0, 0.0, &o.x[k], &o.y[k]);
      o.h[k] = heading_at(R, lid, x0); o.v[k] = sp; o.ts[k] = sp;
      o.lane[k] = o.tgt[k] = closest_lane(R, o.x[k], o.y[k], o.h[k]);
      o.timer[k] = pymod((o.x[k] + o.y[k]) * PI, P->lane_change_delay);
      o.delta[k] = pcg_uniform(&g, cfg->delta_lo, cfg->delta_hi);
    }
  }
  return 0;
}

/* IntersectionEnv._agent_reward / _is_terminated / _is_truncated (intersection_env.py:78-119),
 * has_arrived (:364-369), for the env's controlled vehicle */
/* components (optional, [E][4]): the _agent_rewards dict (intersection_env.py:95-104) in the order
 * collision_reward, high_speed_reward, arrived_reward, on_road_reward. */
int oracle_rewards(const ttrl_state_t* s, const ttrl_lane_table_t* R, const ttrl_reward_cfg_t* cfg,
                   const double* time, float* reward, uint8_t* terminated, uint8_t* truncated, float* components) {
  if (check(s)) return TTRL_E_ARG;
  S o = view(s);
  ttrl_params_t dummy; memset(&dummy, 0, sizeof dummy); dummy.lane_vehicle_length = 5.0;
  for (int e = 0; e < o.E; ++e) {
    const int ei = ego_of(&o, e * o.N);
    if (ei < 0) {
      reward[e] = 0; terminated[e] = 0; truncated[e] = (uint8_t)(time[e] >= cfg->duration);
      if (components) for (int q = 0; q < 4; ++q) components[e * 4 + q] = 0.f;
      continue;
    }
    int k = e * o.N + ei;
    double hs = clipd(lmap(o.v[k], cfg->speed_lo, cfg->speed_hi, 0, 1), 0, 1);
    double sr, rr; local(R, o.lane[k], o.x[k], o.y[k], &sr, &rr);
    int onroad = on_lane(R, &dummy, o.lane[k], sr, rr, 0.0);
    int arrived = R->exit_lane[o.lane[k]] && sr >= cfg->exit_distance;
    double r = cfg->collision_reward * (double)o.crashed[k] + cfg->high_speed_reward * hs +
               cfg->arrived_reward * (double)arrived;
    if (arrived) r = cfg->arrived_reward;
    r *= (double)onroad;
    if (cfg->normalize_reward) r = lmap(r, cfg->collision_reward, cfg->arrived_reward, 0, 1);
    reward[e] = (float)r;
    terminated[e] = (uint8_t)(o.crashed[k] || arrived || (cfg->offroad_terminal && !onroad));
    truncated[e] = (uint8_t)(time[e] >= cfg->duration);
    if (components) {
      components[e * 4 + 0] = (float)o.crashed[k]; components[e * 4 + 1] = (float)hs;
      components[e * 4 + 2] = (float)arrived; components[e * 4 + 3] = (float)onroad;
    }
  }
  return 0;
}

/* ---------------------------------------------------------------- intersection scenario */
static void clear_slot(S* o, int k) {
  o->kind[k] = TTRL_ABSENT; o->crashed[k] = 0; o->hasimp[k] = 0; o->lc[k] = 0;
  o->x[k] = o->y[k] = o->h[k] = o->v[k] = o->ts[k] = o->timer[k] = o->steer[k] = o->acc[k] = 0;
  o->ix[k] = o->iy[k] = 0; o->delta[k] = 4.0; o->lane[k] = o->tgt[k] = 0; o->sidx[k] = -1;
  for (int q = 0; q < TTRL_ROUTE_MAX; ++q) o->rroad[k * TTRL_ROUTE_MAX + q] = o->rlane[k * TTRL_ROUTE_MAX + q] = -1;
  o->rn[k] = -1; o->yield[k] = 0;
}
static void move_slot(S* o, int d, int k) {
  o->kind[d] = o->kind[k]; o->crashed[d] = o->crashed[k]; o->hasimp[d] = o->hasimp[k]; o->lc[d] = o->lc[k];
  o->x[d] = o->x[k]; o->y[d] = o->y[k]; o->h[d] = o->h[k]; o->v[d] = o->v[k]; o->ts[d] = o->ts[k];
  o->timer[d] = o->timer[k]; o->delta[d] = o->delta[k]; o->steer[d] = o->steer[k]; o->acc[d] = o->acc[k];
  o->ix[d] = o->ix[k]; o->iy[d] = o->iy[k]; o->lane[d] = o->lane[k]; o->tgt[d] = o->tgt[k]; o->sidx[d] = o->sidx[k];
  for (int q = 0; q < TTRL_ROUTE_MAX; ++q) {
    o->rroad[d * TTRL_ROUTE_MAX + q] = o->rroad[k * TTRL_ROUTE_MAX + q];
    o->rlane[d * TTRL_ROUTE_MAX + q] = o->rlane[k * TTRL_ROUTE_MAX + q];
  }
  o->rn[d] = o->rn[k]; o->yield[d] = o->yield[k];
}
/* keep[j] for the present slots; survivors move down in list order, the tail is cleared */
static void compact(S* o, int base, const int* keep) {
  int w = 0;
  for (int j = 0; j < o->N; ++j) {
    if (o->kind[base + j] == TTRL_ABSENT || !keep[j]) continue;
    if (w != j) move_slot(o, base + w, base + j);
    w++;
  }
  for (int j = w; j < o->N; ++j) clear_slot(o, base + j);
}
static int count_of(const S* o, int base) {
  int n = 0;
  while (n < o->N && o->kind[base + n] != TTRL_ABSENT) n++;
  return n;
}
/* ControlledVehicle.plan_route_to controller.py:71-87 over RoadNetwork.shortest_path road.py:159-188 */
static void plan_route(S* o, const ttrl_lane_table_t* R, const ttrl_ix_cfg_t* C, int k, int corner) {
  const int l = o->lane[k], road = R->road[l], node = R->road_to[road];
  const int n = C->path_len[node][corner] > 0 ? C->path_len[node][corner] : 0;
  for (int q = 0; q < TTRL_ROUTE_MAX; ++q) o->rroad[k * TTRL_ROUTE_MAX + q] = o->rlane[k * TTRL_ROUTE_MAX + q] = -1;
  o->rroad[k * TTRL_ROUTE_MAX] = (int8_t)road; o->rlane[k * TTRL_ROUTE_MAX] = (int8_t)R->lane_id[l];
  for (int q = 0; q < n; ++q) o->rroad[k * TTRL_ROUTE_MAX + 1 + q] = C->path_road[node][corner][q];
  o->rn[k] = (int8_t)(1 + n);
}
/* IntersectionEnv._spawn_vehicle intersection_env.py:320-348 (IDMVehicle.make_on_lane objects.py:68-89,
 * IDMVehicle.__init__ behavior.py:48-64, randomize_behavior :66-69) */
static void ix_spawn(S* o, const ttrl_lane_table_t* R, const ttrl_params_t* P, const ttrl_ix_cfg_t* C, pcg_t* g,
                     int base, double longitudinal, double pos_dev, double speed_dev, double prob, int go_straight) {
  if (pcg_double(g) > prob) return;
  int route[2];
  pcg_choice_noreplace(g, 4, 2, route);
  if (go_straight) route[1] = (route[0] + 2) % 4;
  const int l = C->entry_lane[route[0]];
  const double lon = longitudinal + C->spawn_offset + pcg_normal(g) * pos_dev;
  const double sp = C->spawn_speed + pcg_normal(g) * speed_dev;
  double px, py;
  position(R, l, lon, 0.0, &px, &py);
  const double ph = heading_at(R, l, lon);
  for (int j = 0; j < o->N; ++j) {
    const int k = base + j;
    if (o->kind[k] == TTRL_ABSENT) continue;
    const double dx = o->x[k] - px, dy = o->y[k] - py;
    if (sqrt(dx * dx + dy * dy) < C->spawn_clear_distance) return;
  }
  const int n = count_of(o, base);
  const double delta = pcg_uniform(g, C->delta_lo, C->delta_hi);  /* drawn even when no slot is left */
  if (n >= o->N) return;
  const int k = base + n;
  clear_slot(o, k);
  o->kind[k] = TTRL_IDM; o->lc[k] = 1;
  o->x[k] = px; o->y[k] = py; o->h[k] = ph; o->v[k] = sp; o->ts[k] = sp;
  o->lane[k] = o->tgt[k] = closest_lane(R, px, py, ph);
  o->timer[k] = pymod((px + py) * PI, P->lane_change_delay);
  plan_route(o, R, C, k, route[1]);
  o->delta[k] = delta;
}
/* IntersectionEnv._clear_vehicles intersection_env.py:350-362 */
static void ix_clear(S* o, const ttrl_lane_table_t* R, const ttrl_ix_cfg_t* C, int base) {
  int keep[256];
  for (int j = 0; j < o->N; ++j) {
    const int k = base + j;
    keep[j] = 1;
    if (o->kind[k] != TTRL_IDM) continue;      /* controlled vehicles stay */
    const int l = o->lane[k];
    double s, r; local(R, l, o->x[k], o->y[k], &s, &r);
    const int leaving = R->exit_lane[l] && s >= R->length[l] - C->leave_margin;
    keep[j] = !(leaving || o->rn[k] < 0);
  }
  compact(o, base, keep);
}

/* IntersectionEnv._reset (intersection_env.py:135-137, _make_vehicles :251-318) from the
 * np_random already seeded in state.rng */
int oracle_ix_reset(const ttrl_state_t* s, const ttrl_lane_table_t* R, const ttrl_params_t* P,
                    const ttrl_ix_cfg_t* C, const uint8_t* mask) {
  if (check(s) || !s->rng || !s->route_n || s->n_veh > 256 || C->initial_vehicle_count > TTRL_IX_MAX_INIT)
    return TTRL_E_ARG;
  S o = view(s);
#pragma omp parallel for schedule(static)
  for (int e = 0; e < o.E; ++e) {
    if (mask && !mask[e]) continue;
    const int base = e * o.N;
    pcg_t g; rng_load(&g, o.rng + (size_t)e * TTRL_RNG_WORDS);
    for (int j = 0; j < o.N; ++j) clear_slot(&o, base + j);
    o.reg[e] = 0;
    for (int t = 0; t < C->initial_vehicle_count - 1; ++t)
      ix_spawn(&o, R, P, C, &g, base, C->init_longitudinal[t], 1.0, 1.0, C->spawn_probability, 0);
    for (int f = 0; f < C->warmup_frames; ++f) {
      act_env(&o, R, P, e);
      step_env(&o, R, P, e, C->warmup_dt);
    }
    ix_spawn(&o, R, P, C, &g, base, C->challenger_longitudinal, C->challenger_position_deviation,
             C->challenger_speed_deviation, 1.0, 1);
    /* the ego MDPVehicle, appended after the traffic (:283-312) */
    const int dest = C->ego_destination >= 0 ? C->ego_destination : 1 + (int)pcg_bounded(&g, 3);
    const double lon = C->ego_longitudinal + C->ego_deviation * (1.0 + pcg_normal(&g));
    int n = count_of(&o, base);
    if (n >= o.N) n = o.N - 1;                   /* no slot left: the last vehicle gives way */
    const int k = base + n;
    clear_slot(&o, k);
    double ex, ey;
    position(R, C->ego_lane, lon, 0.0, &ex, &ey);
    o.kind[k] = TTRL_MDP; o.x[k] = ex; o.y[k] = ey; o.h[k] = heading_at(R, C->ego_lane, C->ego_heading_s);
    o.v[k] = C->ego_speed;
    o.lane[k] = o.tgt[k] = closest_lane(R, ex, ey, o.h[k]);
    o.sidx[k] = speed_to_index(P, C->ego_speed);
    o.ts[k] = P->target_speeds[o.sidx[k]];
    plan_route(&o, R, C, k, dest);
    /* "prevent early collisions": list.remove while iterating skips the next vehicle */
    int lst[256], len = n + 1, keep[256];
    for (int j = 0; j < len; ++j) { lst[j] = j; keep[j] = 1; }
    for (int i = 0; i < len; ++i) {
      const int j = lst[i], kj = base + j;
      const double dx = o.x[kj] - ex, dy = o.y[kj] - ey;
      if (j != n && sqrt(dx * dx + dy * dy) < C->ego_clear_distance) {
        keep[j] = 0;
        for (int q = i; q < len - 1; ++q) lst[q] = lst[q + 1];
        len--;
      }
    }
    compact(&o, base, keep);
    rng_store(&g, o.rng + (size_t)e * TTRL_RNG_WORDS);
  }
  return 0;
}

/* IntersectionEnv.step tail (intersection_env.py:135-139): _clear_vehicles, _spawn_vehicle */
int oracle_ix_clear_spawn(const ttrl_state_t* s, const ttrl_lane_table_t* R, const ttrl_params_t* P,
                          const ttrl_ix_cfg_t* C, const uint8_t* mask) {
  if (check(s) || !s->rng || !s->route_n || s->n_veh > 256) return TTRL_E_ARG;
  S o = view(s);
#pragma omp parallel for schedule(static)
  for (int e = 0; e < o.E; ++e) {
    if (mask && !mask[e]) continue;
    const int base = e * o.N;
    ix_clear(&o, R, C, base);
    pcg_t g; rng_load(&g, o.rng + (size_t)e * TTRL_RNG_WORDS);
    ix_spawn(&o, R, P, C, &g, base, 0.0, 1.0, 1.0, C->spawn_probability, 0);
    rng_store(&g, o.rng + (size_t)e * TTRL_RNG_WORDS);
  }
  return 0;
}

/* numpy Generator draws, exposed for tests/test_ix_rng.py: op 0 standard_normal, 1 random,
 * 2 integers(0, arg), 3 choice(arg, 2, replace=False) (2 outputs), 4 shuffle of arg rows
 * (arg outputs: the permutation); one output slot per value */
int oracle_rng_ops(uint64_t* state5, const int32_t* ops, const int32_t* args, int32_t n_ops, double* out) {
  pcg_t g; rng_load(&g, state5);
  int w = 0;
  for (int i = 0; i < n_ops; ++i) {
    switch (ops[i]) {
      case 0: out[w++] = pcg_normal(&g); break;
      case 1: out[w++] = pcg_double(&g); break;
      case 2: out[w++] = (double)pcg_bounded(&g, (uint32_t)args[i]); break;
      case 3: { int r[2]; pcg_choice_noreplace(&g, args[i], 2, r); out[w++] = r[0]; out[w++] = r[1]; break; }
      case 4: {
        int perm[256]; const int n = args[i];
        for (int t = 0; t < n; ++t) perm[t] = t;
        for (int t = n - 1; t >= 1; --t) { const int j = (int)pcg_interval(&g, (uint64_t)t); const int u = perm[t]; perm[t] = perm[j]; perm[j] = u; }
        for (int t = 0; t < n; ++t) out[w++] = perm[t];
        break;
      }
      default: return TTRL_E_ARG;
    }
  }
  rng_store(&g, state5);
  return w;
}

/* ---------------------------------------------------------------------------------------
 * TimeToCollisionObservation (observation.py:114-151) over compute_ttc_grid
 * (finite_mdp.py:104-167), on the single straight road: every vehicle is on the ego's road
 * with the same lane count, so `lane = [other.lane_index[2]]` (finite_mdp.py:142-149).
 */
/* margin (optional, shaped as out): a contribution's decisions -- the equal-speed skip, the sign
 * of the time to collision (distance and closing speed, not_zero's switch), its bin (int() and
 * ceil of t / quantization) and the horizon test -- recorded into the bins around its time. */
int oracle_observe_ttc_m(const ttrl_state_t* s, const ttrl_lane_table_t* R, const ttrl_params_t* P,
                         const ttrl_ttc_cfg_t* cfg, float* out, double* margin) {
  if (check(s) || !cfg || !out) return TTRL_E_ARG;
  S o = view(s);
  const int NS = P->n_target_speeds, NL = R->n_lanes, T = cfg->horizon_bins;
  const int OL = cfg->obs_lanes, OS = cfg->obs_speeds;
  const int raw = OS == 0 && OL == 0;
  if (margin)
    for (size_t q = 0; q < (size_t)o.E * (raw ? NS * NL : OS * OL) * T; ++q) margin[q] = INFINITY;
#pragma omp parallel
  {
  double* grid = (double*)malloc(sizeof(double) * NS * NL * T);
  double* gm = (double*)malloc(sizeof(double) * NS * NL * T);
#pragma omp for schedule(static)
  for (int e = 0; e < o.E; ++e) {
    const int base = e * o.N, ego = base;
    for (int k = 0; k < NS * NL * T; ++k) { grid[k] = 0; gm[k] = INFINITY; }
    const double ec = cos(o.h[ego]), es = sin(o.h[ego]);
    for (int si = 0; si < NS; ++si) {
      const double ego_speed = P->target_speeds[si];             /* index_to_speed controller.py:317-324 */
      for (int j = 0; j < o.N; ++j) {                             /* env.road.vehicles, list order */
        const int k = base + j;
        if (j == 0 || o.kind[k] == TTRL_ABSENT) continue;
        const double m_eq = fabs(ego_speed - o.v[k]) / (1 + fabs(ego_speed));
        if (ego_speed == o.v[k] && !margin) continue;
        const double margin_len = P->length / 2 + P->length / 2;
        const double pts[3][2] = {{0, 1}, {-margin_len, 0.5}, {margin_len, 0.5}};
        for (int c = 0; c < 3; ++c) {
          const double distance = lane_distance(&o, R, base, 0, j) + pts[c][0];
          const double proj = o.v[k] * (cos(o.h[k]) * ec + sin(o.h[k]) * es);
          const double ttc = distance / not_zero(ego_speed - proj);
          const int l = o.lane[k];
          const double q = ttc / cfg->time_quantization;
          if (margin) {
            const double den = ego_speed - proj, sc = 1 + fabs(ego_speed) + fabs(proj);
            double m = m_eq;
            const double pos = 1 + fabs(o.x[k]) + fabs(o.y[k]) + fabs(o.x[ego]) + fabs(o.y[ego]);
            if (fabs(distance) / pos < m) m = fabs(distance) / pos;
            if (fabs(den) / sc < m) m = fabs(den) / sc;
            if (fabs(fabs(den) - 1e-2) / sc < m) m = fabs(fabs(den) - 1e-2) / sc;
            const double aq = fabs(q), fq = aq - floor(aq);
            const double mq = (fq < 0.5 ? fq : 1 - fq) / (1 + aq);
            if (mq < m) m = mq;
            if (fabs(T - aq) / (1 + aq) < m) m = fabs(T - aq) / (1 + aq);
            for (double t = floor(aq) - 1; t <= ceil(aq) + 1; ++t)
              if (0 <= t && t < T) {
                double* g = &gm[(si * NL + l) * T + (int)t];
                if (m < *g) *g = m;
              }
          }
          if (ego_speed == o.v[k]) continue;
          if (ttc < 0) continue;
          const double times[2] = {q, ceil(q)};                   /* int() of a non-negative value */
          for (int u = 0; u < 2; ++u) {
            if (!(times[u] < (double)T)) continue;
            const int t = (int)times[u];
            double* g = &grid[(si * NL + l) * T + t];
            if (pts[c][1] > *g) *g = pts[c][1];                    /* np.maximum */
          }
        }
      }
    }
    if (OS == 0 && OL == 0) {                                     /* raw grid (finite_mdp.py:48) */
      for (int k = 0; k < NS * NL * T; ++k) out[(size_t)e * NS * NL * T + k] = (float)grid[k];
      if (margin)
        for (int k = 0; k < NS * NL * T; ++k) margin[(size_t)e * NS * NL * T + k] = gm[k];
      continue;
    }
    /* observation.py:136-151: pad lanes with ones, window of obs_lanes around the ego's
     * lane; repeat the first / last speed rows (1 + NS) times, window of obs_speeds */
    const int lane = o.lane[ego], sidx = o.sidx[ego];
    float* ob = out + (size_t)e * OS * OL * T;
    for (int a = 0; a < OS; ++a) {
      const int row = NS + sidx - OS / 2 + a;                      /* row of the repeated array */
      int sp = row < 1 + NS ? 0 : (row >= 2 * NS ? NS - 1 : row - NS);
      for (int b = 0; b < OL; ++b) {
        const int l = lane - OL / 2 + b;
        for (int t = 0; t < T; ++t) {
          ob[(a * OL + b) * T + t] = (l < 0 || l >= NL) ? 1.0f : (float)grid[(sp * NL + l) * T + t];
          if (margin)
            margin[(size_t)e * OS * OL * T + (a * OL + b) * T + t] = (l < 0 || l >= NL) ? INFINITY
                                                                                       : gm[(sp * NL + l) * T + t];
        }
      }
    }
  }
  free(grid);
  free(gm);
  }
  return TTRL_OK;
}

int oracle_observe_ttc(const ttrl_state_t* s, const ttrl_lane_table_t* R, const ttrl_params_t* P,
                       const ttrl_ttc_cfg_t* cfg, float* out) {
  return oracle_observe_ttc_m(s, R, P, cfg, out, NULL);
}

/* utils.distance_to_rect utils.py:386-413 for the ray [r, q] and rectangle corners a, b, c, d */
static double distance_to_rect(const double r[2], const double q[2], double c[4][2]) {
  double ux = c[1][0] - c[0][0], uy = c[1][1] - c[0][1], vx = c[3][0] - c[0][0], vy = c[3][1] - c[0][1];
  const double nu = sqrt(ux * ux + uy * uy), nv = sqrt(vx * vx + vy * vy);
  ux /= nu; uy /= nu; vx /= nv; vy /= nv;
  const double qrx = q[0] - r[0], qry = q[1] - r[1];
  const double rqu = qrx * ux + qry * uy, rqv = qrx * vx + qry * vy;
  double i1[2] = {((c[0][0] - r[0]) * ux + (c[0][1] - r[1]) * uy) / rqu,
                  ((c[1][0] - r[0]) * ux + (c[1][1] - r[1]) * uy) / rqu};
  double i2[2] = {((c[0][0] - r[0]) * vx + (c[0][1] - r[1]) * vy) / rqv,
                  ((c[3][0] - r[0]) * vx + (c[3][1] - r[1]) * vy) / rqv};
  if (!(rqu >= 0)) { const double t = i1[0]; i1[0] = i1[1]; i1[1] = t; }
  if (!(rqv >= 0)) { const double t = i2[0]; i2[0] = i2[1]; i2[1] = t; }
  if (interval_distance(i1[0], i1[1], i2[0], i2[1]) <= 0 && interval_distance(0, 1, i1[0], i1[1]) <= 0 &&
      interval_distance(0, 1, i2[0], i2[1]) <= 0)
    return (i1[0] > i2[0] ? i1[0] : i2[0]) * sqrt(qrx * qrx + qry * qry);
  return INFINITY;
}

static int angle_to_index(double angle, double step, int cells) {  /* observation.py:761-762 */
  long k = (long)floor(angle / step) % cells;
  return (int)(k < 0 ? k + cells : k);
}

/* The ray index of an angle (angle_to_index) and its margin: the arc length in metres, at
 * `dist` from the observer, to the nearer sector boundary, relative to `scale`. */
static double ray_mg(double angle, double step, double dist, double scale) {
  const double u = angle / step, f = u - floor(u);
  return (f < 0.5 ? f : 1 - f) * step * dist / scale;
}
static void mg_rays(double* m, int C, int from, int to, double v) {  /* rays from..to (wrapping), +-1 */
  if (!m) return;
  const int n = ((to - from) % C + C) % C + 3;
  for (int u = 0; u < n && u < C; ++u) mg_cell(m, (size_t)(((from - 1 + u) % C + C) % C), v);
}

/* LidarObservation.trace observation.py:704-752 (obstacles: the other vehicles, list order);
 * margin (optional, [E][cells]): each ray's decisions -- a vehicle's range test, the sector of its
 * centre and of its corners' angular extent, the ray-rectangle hit test, and the nearest-hit
 * comparison between vehicles. */
int oracle_observe_lidar_m(const ttrl_state_t* s, const ttrl_lane_table_t* R, const ttrl_params_t* P,
                           const ttrl_lidar_cfg_t* cfg, float* out, double* margin) {
  (void)R;
  if (check(s) || !cfg || !out || cfg->cells < 1 || cfg->cells > 64) return TTRL_E_ARG;
  S o = view(s);
  const int C = cfg->cells;
  const double range = cfg->maximum_range, step = 2 * PI / C;
  if (margin)
    for (size_t q = 0; q < (size_t)o.E * C; ++q) margin[q] = INFINITY;
#pragma omp parallel for schedule(static)
  for (int e = 0; e < o.E; ++e) {
    const int base = e * o.N, ei = ego_of(&o, base), ego = base + ei;
    double grid[64][2];
    double best2[64][2];  /* the two smallest hit distances of each ray, for the comparison margin */
    int who[64];
    double* rm = margin ? margin + (size_t)e * C : NULL;
    for (int c = 0; c < C; ++c) { grid[c][0] = grid[c][1] = range; best2[c][0] = best2[c][1] = INFINITY; who[c] = -1; }
    if (ei < 0) {
      for (int c = 0; c < C; ++c) out[(size_t)e * C * 2 + 2 * c] = out[(size_t)e * C * 2 + 2 * c + 1] = (float)(cfg->normalize ? 1.0 : range);
      continue;
    }
    const double ox = o.x[ego], oy = o.y[ego];
    const double ovx = o.v[ego] * cos(o.h[ego]), ovy = o.v[ego] * sin(o.h[ego]);
    for (int j = 0; j < o.N; ++j) {
      const int k = base + j;
      if (j == ei || o.kind[k] == TTRL_ABSENT) continue;
      const double dx = o.x[k] - ox, dy = o.y[k] - oy;
      const double center_distance = sqrt(dx * dx + dy * dy);
      const double scale = 1 + fabs(o.x[k]) + fabs(o.y[k]) + fabs(ox) + fabs(oy);
      const double m_range = fabs(center_distance - range) / scale;
      if (center_distance > range) {
        if (rm && m_range < 1e-3) mg_rays(rm, C, 0, C - 1, m_range);  /* at the range: any of its rays */
        continue;
      }
      const double vx = o.v[k] * cos(o.h[k]) - ovx, vy = o.v[k] * sin(o.h[k]) - ovy;
      const int ci = angle_to_index(atan2(dy, dx) + step / 2, step, C);
      const double distance = center_distance - P->width / 2;
      if (rm) {
        mg_rays(rm, C, ci, ci, ray_mg(atan2(dy, dx) + step / 2, step, center_distance, scale));
        if (m_range < 1e-3) mg_rays(rm, C, 0, C - 1, m_range);
      }
#define HIT(c_, d_)                                                                               \
  do {                                                                                            \
    if (who[c_] != j) {                                                                           \
      if ((d_) < best2[c_][0]) { best2[c_][1] = best2[c_][0]; best2[c_][0] = (d_); who[c_] = j; } \
      else if ((d_) < best2[c_][1]) best2[c_][1] = (d_);                                          \
    } else if ((d_) < best2[c_][0]) best2[c_][0] = (d_);                                          \
  } while (0)
      HIT(ci, distance);
      if (distance <= grid[ci][0]) {
        grid[ci][0] = distance;
        grid[ci][1] = vx * cos(ci * step) + vy * sin(ci * step);
      }
      /* utils.rect_corners utils.py:126-155: rotation @ corners + center */
      const double hl = P->length / 2, hw = P->width / 2, c = cos(o.h[k]), sn = sin(o.h[k]);
      const double lc[4][2] = {{-hl, -hw}, {-hl, hw}, {hl, hw}, {hl, -hw}};
      double corners[4][2];
      double amin = 0, amax = 0;
      for (int q = 0; q < 4; ++q) {
        corners[q][0] = c * lc[q][0] + (-sn) * lc[q][1] + o.x[k];
        corners[q][1] = sn * lc[q][0] + c * lc[q][1] + o.y[k];
        const double a = atan2(corners[q][1] - oy, corners[q][0] - ox) + step / 2;
        if (q == 0 || a < amin) amin = a;
        if (q == 0 || a > amax) amax = a;
      }
      if (amin < -PI / 2 && -PI / 2 < PI / 2 && PI / 2 < amax) {  /* corners wrap around +pi */
        const double t = amin;
        amin = amax;
        amax = t + 2 * PI;
      }
      const int start = angle_to_index(amin, step, C), end = angle_to_index(amax, step, C);
      const int n = start < end ? end - start + 1 : (C - start) + end + 1;
      if (rm) {  /* the corners' sectors, the wrap test: the vehicle's whole span of rays */
        double m = ray_mg(amin, step, center_distance, scale);
        const double m2 = ray_mg(amax, step, center_distance, scale);
        if (m2 < m) m = m2;
        const double mw = fmin(fabs(amin + PI / 2), fabs(amax - PI / 2)) * center_distance / scale;
        if (mw < m) m = mw;
        mg_rays(rm, C, start, end, m);
      }
      for (int u = 0; u < n; ++u) {
        const int idx = start < end ? start + u : (u < C - start ? start + u : u - (C - start));
        const double dirx = cos(idx * step), diry = sin(idx * step);
        const double r[2] = {ox, oy}, qq[2] = {ox + range * dirx, oy + range * diry};
        const double d = distance_to_rect(r, qq, corners);
        if (rm) {  /* the hit test: the ray's distance to the rectangle's nearest edge line */
          double mh = INFINITY;
          for (int q = 0; q < 4; ++q) {  /* the corners' signed distances to the ray's line */
            const double cd = fabs((corners[q][0] - ox) * diry - (corners[q][1] - oy) * dirx);
            if (cd / scale < mh) mh = cd / scale;
          }
          mg_cell(rm, (size_t)idx, mh);
        }
        if (d < INFINITY) HIT(idx, d);
        if (d <= grid[idx][0]) {
          grid[idx][0] = d;
          grid[idx][1] = vx * dirx + vy * diry;
        }
      }
    }
#undef HIT
    if (rm)  /* the nearest hit of each ray against the runner-up vehicle's */
      for (int c = 0; c < C; ++c)
        if (best2[c][1] < INFINITY) mg_cell(rm, (size_t)c, fabs(best2[c][1] - best2[c][0]) / (1 + range));
    float* ob = out + (size_t)e * C * 2;
    for (int c = 0; c < C; ++c) {
      ob[2 * c] = (float)(cfg->normalize ? grid[c][0] / range : grid[c][0]);
      ob[2 * c + 1] = (float)(cfg->normalize ? grid[c][1] / range : grid[c][1]);
    }
  }
  return TTRL_OK;
}

int oracle_observe_lidar(const ttrl_state_t* s, const ttrl_lane_table_t* R, const ttrl_params_t* P,
                         const ttrl_lidar_cfg_t* cfg, float* out) {
  return oracle_observe_lidar_m(s, R, P, cfg, out, NULL);
}
