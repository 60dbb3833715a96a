// ttrl_torch_ops.cpp — the C ABI of include/ttrl_mi355x.h registered as PyTorch operators
// (torch.ops.ttrl.*), SURVEY.md §8(b) "Native ops".
//
// Every device entry point of libttrl_mi355x.so is one operator here.  The ops are thin: they
// check the tensors, take the current HIP stream of the state's device, allocate their outputs
// from the caching allocator and call the C ABI, which enqueues the kernels.  Nothing here
// computes; there is no CPU kernel (the oracle is test infrastructure and is never dispatched to).
//
// Arguments common to the ops:
//   state   the 24 BatchState tensors in _abi.ALL_FIELDS order (ttrl_state_t field order): 11 real
//           fields (float32 / float64), lane, target_lane, speed_index (int32), kind, crashed,
//           has_impact, lane_change (uint8), route_road, route_lane, route_n (int8), yielding
//           (uint8), reg_steps (int32 [E]), rng (int64 [E][5]); all on one HIP device.
//   lanes / params / cfg   the ABI structs (ttrl_lane_table_t, ttrl_params_t, ttrl_*_cfg_t) as
//           uint8 CPU tensors holding their exact bytes (ops.struct_tensor).
// Schemas mark what an op mutates (Tensor(a!)); Meta kernels give shapes only.
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include <cstddef>
#include <cstring>

#include "ttrl_mi355x.h"

namespace {

constexpr int kFields = 24;  // _abi.ALL_FIELDS

template <typename T>
const T* as_struct(const at::Tensor& t, const char* what) {
  TORCH_CHECK(t.device().is_cpu() && t.scalar_type() == at::kByte && t.is_contiguous() &&
                  t.numel() == static_cast<int64_t>(sizeof(T)),
              "ttrl: ", what, " must be a ", sizeof(T), "-byte uint8 CPU tensor (ops.struct_tensor)");
  return reinterpret_cast<const T*>(t.data_ptr());
}

void* ptr(const at::Tensor& t) { return t.defined() && t.numel() ? t.data_ptr() : nullptr; }

// ttrl_state_t over the state tensor list (pointers in ALL_FIELDS order).
ttrl_state_t state_of(at::TensorList ts) {
  TORCH_CHECK(ts.size() == kFields, "ttrl: state must hold ", kFields, " tensors in _abi.ALL_FIELDS order, got ",
              ts.size());
  const at::Tensor& x = ts[0];
  TORCH_CHECK(x.dim() == 2, "ttrl: state tensors are [n_envs, n_veh]");
  TORCH_CHECK(x.scalar_type() == at::kDouble || x.scalar_type() == at::kFloat, "ttrl: real fields are float32/64");
  const auto dev = x.device();
  for (const auto& t : ts) {
    TORCH_CHECK(t.device() == dev, "ttrl: every state tensor must live on ", dev);
    TORCH_CHECK(t.is_contiguous(), "ttrl: state tensors must be contiguous");
  }
  for (int i = 0; i < 11; ++i)
    TORCH_CHECK(ts[i].scalar_type() == x.scalar_type() && ts[i].sizes() == x.sizes(), "ttrl: real field ", i,
                " must match x");
  ttrl_state_t s;
  std::memset(&s, 0, sizeof(s));
  s.n_envs = static_cast<int32_t>(x.size(0));
  s.n_veh = static_cast<int32_t>(x.size(1));
  s.dtype = x.scalar_type() == at::kDouble ? TTRL_F64 : TTRL_F32;
  // the 24 field pointers follow the 4 int32 header words, in ALL_FIELDS order
  static_assert(offsetof(ttrl_state_t, rng) - offsetof(ttrl_state_t, x) == (kFields - 1) * sizeof(void*),
                "ttrl_state_t: the field pointers must be contiguous");
  char* base = reinterpret_cast<char*>(&s) + offsetof(ttrl_state_t, x);
  for (int i = 0; i < kFields; ++i) {
    void* p = ts[i].data_ptr();
    std::memcpy(base + i * sizeof(void*), &p, sizeof(void*));
  }
  return s;
}

void check_hip(const at::Tensor& t) {
  TORCH_CHECK(t.device().is_cuda(), "ttrl ops run on a HIP device only (no CPU fallback), got ", t.device());
}

hipStream_t stream_of(const at::Tensor& t) { return c10::hip::getCurrentHIPStream(t.device().index()).stream(); }

void ok(int rc, const char* name) {
  TORCH_CHECK(rc == 0, "ttrl: ", name, " failed: ",
              rc == TTRL_E_ARG ? "TTRL_E_ARG (bad argument)"
                               : rc == TTRL_E_LAUNCH ? "TTRL_E_LAUNCH (HIP error)" : "TTRL_E_UNSUPPORTED");
}

at::Tensor dev_i32(const c10::optional<at::Tensor>& t, int64_t n, const at::Tensor& like, const char* what) {
  if (!t || !t->defined()) return at::Tensor();
  at::Tensor a = t->to(like.device(), at::kInt).contiguous();
  TORCH_CHECK(a.numel() == n, "ttrl: ", what, " needs ", n, " entries, got ", a.numel());
  return a;
}

at::Tensor dev_u8(const c10::optional<at::Tensor>& t, int64_t n, const at::Tensor& like, const char* what) {
  if (!t || !t->defined()) return at::Tensor();
  at::Tensor a = t->to(like.device(), at::kByte).contiguous();
  TORCH_CHECK(a.numel() == n, "ttrl: ", what, " needs ", n, " entries, got ", a.numel());
  return a;
}

at::TensorOptions opts(const at::Tensor& like, at::ScalarType dt) { return like.options().dtype(dt); }

// ------------------------------------------------------------------------------------ frame ops
void simulate_(at::TensorList state, const at::Tensor& lanes, const at::Tensor& params,
               const c10::optional<at::Tensor>& actions, int64_t frames, double dt) {
  check_hip(state[0]);
  ttrl_state_t s = state_of(state);
  at::Tensor a = dev_i32(actions, s.n_envs, state[0], "actions");
  ok(ttrl_simulate(&s, as_struct<ttrl_lane_table_t>(lanes, "lanes"), as_struct<ttrl_params_t>(params, "params"),
                   static_cast<const int32_t*>(ptr(a)), static_cast<int32_t>(frames), dt, stream_of(state[0])),
     "ttrl_simulate");
}

void road_act_(at::TensorList state, const at::Tensor& lanes, const at::Tensor& params) {
  check_hip(state[0]);
  ttrl_state_t s = state_of(state);
  ok(ttrl_road_act(&s, as_struct<ttrl_lane_table_t>(lanes, "lanes"), as_struct<ttrl_params_t>(params, "params"),
                   stream_of(state[0])),
     "ttrl_road_act");
}

void road_step_(at::TensorList state, const at::Tensor& lanes, const at::Tensor& params, double dt) {
  check_hip(state[0]);
  ttrl_state_t s = state_of(state);
  ok(ttrl_road_step(&s, as_struct<ttrl_lane_table_t>(lanes, "lanes"), as_struct<ttrl_params_t>(params, "params"),
                    dt, stream_of(state[0])),
     "ttrl_road_step");
}

void meta_action_(at::TensorList state, const at::Tensor& lanes, const at::Tensor& params,
                  const at::Tensor& actions) {
  check_hip(state[0]);
  ttrl_state_t s = state_of(state);
  at::Tensor a = dev_i32(actions, s.n_envs, state[0], "actions");
  ok(ttrl_meta_action(&s, as_struct<ttrl_lane_table_t>(lanes, "lanes"), as_struct<ttrl_params_t>(params, "params"),
                      static_cast<const int32_t*>(ptr(a)), stream_of(state[0])),
     "ttrl_meta_action");
}

// The whole env.step (AbstractEnv.step abstract.py:224-250) in one launch: the fused frames, the
// Kinematics observation of the final state (kin_cfg given; else obs / ids are empty) and the step
// tail (time += time_inc, reward, terminated, truncated, components, the info's ego speed / crashed).
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor>
env_step_outputs(const at::Tensor& x, const ttrl_kin_cfg_t* kc, const ttrl_grid_cfg_t* gc = nullptr) {
  const int64_t E = x.size(0);
  at::Tensor obs, ids;
  if (gc) {
    obs = at::empty({E, gc->n_features, gc->shape_x, gc->shape_y}, opts(x, at::kFloat));
    ids = at::empty({0}, opts(x, at::kInt));
  } else if (kc) {
    obs = at::empty({E, kc->vehicles_count, kc->n_features}, opts(x, at::kFloat));
    ids = at::empty({E, std::max<int64_t>(kc->vehicles_count - 1, 1)}, opts(x, at::kInt));
  } else {
    obs = at::empty({0}, opts(x, at::kFloat));
    ids = at::empty({0}, opts(x, at::kInt));
  }
  return {obs, ids, at::empty({E}, opts(x, at::kFloat)), at::empty({E}, opts(x, at::kBool)),
          at::empty({E}, opts(x, at::kBool)), at::empty({E, 4}, opts(x, at::kFloat)),
          at::empty({E}, opts(x, x.scalar_type())), at::empty({E}, opts(x, at::kBool))};
}

std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor> env_step_(
    at::TensorList state, const at::Tensor& lanes, const at::Tensor& params, const c10::optional<at::Tensor>& actions,
    int64_t frames, double dt, const c10::optional<at::Tensor>& kin_cfg, const at::Tensor& reward_cfg,
    const at::Tensor& time, double time_inc, const c10::optional<at::Tensor>& order,
    at::OptionalIntArrayRef action_lut, const c10::optional<at::Tensor>& grid_cfg) {
  check_hip(state[0]);
  ttrl_state_t s = state_of(state);
  const ttrl_kin_cfg_t* kc = kin_cfg && kin_cfg->defined() ? as_struct<ttrl_kin_cfg_t>(*kin_cfg, "kin_cfg") : nullptr;
  const ttrl_grid_cfg_t* gc =
      grid_cfg && grid_cfg->defined() ? as_struct<ttrl_grid_cfg_t>(*grid_cfg, "grid_cfg") : nullptr;
  TORCH_CHECK(!(kc && gc), "ttrl: env_step_ takes a kin_cfg or a grid_cfg, not both");
  TORCH_CHECK(time.device() == state[0].device() && time.scalar_type() == at::kDouble && time.is_contiguous() &&
                  time.numel() == s.n_envs,
              "ttrl: time must be a contiguous float64 [n_envs] tensor on the state's device");
  at::Tensor a = dev_i32(actions, s.n_envs, state[0], "actions");
  const bool od = order && order->defined();
  if (od)  // a permutation of the envs (its first n_envs entries; ix_step_tail_'s buffer is 2 n_envs)
    TORCH_CHECK(order->device() == state[0].device() && order->scalar_type() == at::kInt && order->is_contiguous() &&
                    order->numel() >= s.n_envs,
                "ttrl: order must be a contiguous int32 tensor of at least n_envs entries on the state's device");
  std::vector<int32_t> lut;  // the action index -> meta-action code table (host; ttrl_env_step copies it)
  if (action_lut.has_value())
    for (int64_t c : *action_lut) lut.push_back(static_cast<int32_t>(c));
  auto out = env_step_outputs(state[0], kc, gc);
  auto& [obs, ids, rew, term, trunc, comp, speed, crashed] = out;
  if (gc) {  // the OccupancyGrid of the final state (the step's own launch where it fuses)
    TORCH_CHECK(!od, "ttrl: env_step_ with a grid_cfg takes no dispatch order (straight roads)");
    ok(ttrl_env_step_grid(&s, as_struct<ttrl_lane_table_t>(lanes, "lanes"), as_struct<ttrl_params_t>(params, "params"),
                          static_cast<const int32_t*>(ptr(a)), static_cast<int32_t>(frames), dt, gc,
                          obs.data_ptr<float>(), as_struct<ttrl_reward_cfg_t>(reward_cfg, "reward_cfg"),
                          time.data_ptr<double>(), time_inc, rew.data_ptr<float>(),
                          static_cast<uint8_t*>(term.data_ptr()), static_cast<uint8_t*>(trunc.data_ptr()),
                          comp.data_ptr<float>(), speed.data_ptr(), static_cast<uint8_t*>(crashed.data_ptr()),
                          lut.empty() ? nullptr : lut.data(), static_cast<int32_t>(lut.size()), stream_of(state[0])),
       "ttrl_env_step_grid");
    return out;
  }
  ok(ttrl_env_step(&s, as_struct<ttrl_lane_table_t>(lanes, "lanes"), as_struct<ttrl_params_t>(params, "params"),
                   static_cast<const int32_t*>(ptr(a)), static_cast<int32_t>(frames), dt, kc,
                   kc ? obs.data_ptr<float>() : nullptr, kc ? ids.data_ptr<int32_t>() : nullptr,
                   as_struct<ttrl_reward_cfg_t>(reward_cfg, "reward_cfg"), time.data_ptr<double>(), time_inc,
                   rew.data_ptr<float>(), static_cast<uint8_t*>(term.data_ptr()),
                   static_cast<uint8_t*>(trunc.data_ptr()), comp.data_ptr<float>(), speed.data_ptr(),
                   static_cast<uint8_t*>(crashed.data_ptr()), od ? order->data_ptr<int32_t>() : nullptr,
                   lut.empty() ? nullptr : lut.data(), static_cast<int32_t>(lut.size()), stream_of(state[0])),
     "ttrl_env_step");
  return out;
}

std::tuple<at::Tensor, at::Tensor> neighbours(at::TensorList state, const at::Tensor& lanes,
                                              const c10::optional<at::Tensor>& query_lane) {
  check_hip(state[0]);
  ttrl_state_t s = state_of(state);
  at::Tensor q = dev_i32(query_lane, int64_t(s.n_envs) * s.n_veh, state[0], "query_lane");
  at::Tensor f = at::empty({s.n_envs, s.n_veh}, opts(state[0], at::kInt)), r = at::empty_like(f);
  ok(ttrl_neighbours(&s, as_struct<ttrl_lane_table_t>(lanes, "lanes"), static_cast<const int32_t*>(ptr(q)),
                     f.data_ptr<int32_t>(), r.data_ptr<int32_t>(), stream_of(state[0])),
     "ttrl_neighbours");
  return {f, r};
}

// ------------------------------------------------------------------------------------ observers
std::tuple<at::Tensor, at::Tensor> kin_outputs(const at::Tensor& x, const ttrl_kin_cfg_t* c) {
  const int64_t E = x.size(0);
  // one observed vehicle (the ego alone) has no id column: the kernels write none, so the
  // placeholder column holds the padding id -1 instead of uninitialised memory
  const int64_t w = std::max<int64_t>(c->vehicles_count - 1, 1);
  return {at::empty({E, c->vehicles_count, c->n_features}, opts(x, at::kFloat)),
          c->vehicles_count > 1 ? at::empty({E, w}, opts(x, at::kInt)) : at::full({E, w}, -1, opts(x, at::kInt))};
}

std::tuple<at::Tensor, at::Tensor> kinematics_obs(at::TensorList state, const at::Tensor& lanes,
                                                  const at::Tensor& params, const at::Tensor& cfg) {
  check_hip(state[0]);
  ttrl_state_t s = state_of(state);
  const auto* c = as_struct<ttrl_kin_cfg_t>(cfg, "cfg");
  auto [out, ids] = kin_outputs(state[0], c);
  ok(ttrl_observe_kinematics(&s, as_struct<ttrl_lane_table_t>(lanes, "lanes"),
                             as_struct<ttrl_params_t>(params, "params"), c, out.data_ptr<float>(),
                             ids.data_ptr<int32_t>(), stream_of(state[0])),
     "ttrl_observe_kinematics");
  return {out, ids};
}

void kinematics_obs_masked_(at::TensorList state, const at::Tensor& lanes, const at::Tensor& params,
                            const at::Tensor& cfg, const at::Tensor& mask, const at::Tensor& out,
                            const at::Tensor& ids) {
  check_hip(state[0]);
  ttrl_state_t s = state_of(state);
  const auto* c = as_struct<ttrl_kin_cfg_t>(cfg, "cfg");
  at::Tensor m = dev_u8(mask, s.n_envs, state[0], "mask");
  TORCH_CHECK(out.is_contiguous() && out.scalar_type() == at::kFloat &&
                  out.numel() == int64_t(s.n_envs) * c->vehicles_count * c->n_features,
              "ttrl: out must be a contiguous float32 [E, V, F] tensor");
  TORCH_CHECK(ids.is_contiguous() && ids.scalar_type() == at::kInt &&
                  ids.numel() == int64_t(s.n_envs) * std::max(c->vehicles_count - 1, 1),
              "ttrl: ids must be a contiguous int32 [E, V-1] tensor");
  ok(ttrl_observe_kinematics_masked(&s, as_struct<ttrl_lane_table_t>(lanes, "lanes"),
                                    as_struct<ttrl_params_t>(params, "params"), c,
                                    static_cast<const uint8_t*>(ptr(m)), out.data_ptr<float>(),
                                    ids.data_ptr<int32_t>(), stream_of(state[0])),
     "ttrl_observe_kinematics_masked");
}

at::Tensor occupancy_grid(at::TensorList state, const at::Tensor& lanes, const at::Tensor& params,
                          const at::Tensor& cfg) {
  check_hip(state[0]);
  ttrl_state_t s = state_of(state);
  const auto* c = as_struct<ttrl_grid_cfg_t>(cfg, "cfg");
  at::Tensor out = at::empty({s.n_envs, c->n_features, c->shape_x, c->shape_y}, opts(state[0], at::kFloat));
  ok(ttrl_observe_grid(&s, as_struct<ttrl_lane_table_t>(lanes, "lanes"), as_struct<ttrl_params_t>(params, "params"),
                       c, out.data_ptr<float>(), stream_of(state[0])),
     "ttrl_observe_grid");
  return out;
}

std::vector<int64_t> ttc_shape(int64_t E, const ttrl_lane_table_t* R, const ttrl_params_t* P,
                               const ttrl_ttc_cfg_t* c) {
  if (c->obs_speeds == 0 && c->obs_lanes == 0) return {E, P->n_target_speeds, R->n_lanes, c->horizon_bins};
  return {E, c->obs_speeds, c->obs_lanes, c->horizon_bins};
}

at::Tensor observe_ttc(at::TensorList state, const at::Tensor& lanes, const at::Tensor& params,
                       const at::Tensor& cfg) {
  check_hip(state[0]);
  ttrl_state_t s = state_of(state);
  const auto* R = as_struct<ttrl_lane_table_t>(lanes, "lanes");
  const auto* P = as_struct<ttrl_params_t>(params, "params");
  const auto* c = as_struct<ttrl_ttc_cfg_t>(cfg, "cfg");
  at::Tensor out = at::empty(ttc_shape(s.n_envs, R, P, c), opts(state[0], at::kFloat));
  ok(ttrl_observe_ttc(&s, R, P, c, out.data_ptr<float>(), stream_of(state[0])), "ttrl_observe_ttc");
  return out;
}

at::Tensor observe_lidar(at::TensorList state, const at::Tensor& lanes, const at::Tensor& params,
                         const at::Tensor& cfg) {
  check_hip(state[0]);
  ttrl_state_t s = state_of(state);
  const auto* c = as_struct<ttrl_lidar_cfg_t>(cfg, "cfg");
  at::Tensor out = at::empty({s.n_envs, c->cells, 2}, opts(state[0], at::kFloat));
  ok(ttrl_observe_lidar(&s, as_struct<ttrl_lane_table_t>(lanes, "lanes"), as_struct<ttrl_params_t>(params, "params"),
                        c, out.data_ptr<float>(), stream_of(state[0])),
     "ttrl_observe_lidar");
  return out;
}

// ------------------------------------------------------------------------------------ resets
void reset_highway_(at::TensorList state, const at::Tensor& lanes, const at::Tensor& params, const at::Tensor& cfg,
                    const at::Tensor& pcg) {
  check_hip(state[0]);
  ttrl_state_t s = state_of(state);
  TORCH_CHECK(pcg.device() == state[0].device() && pcg.scalar_type() == at::kLong && pcg.is_contiguous() &&
                  pcg.numel() == int64_t(s.n_envs) * 4,
              "ttrl: pcg must be a contiguous int64 [n_envs, 4] tensor on the state's device");
  ok(ttrl_reset_highway(&s, as_struct<ttrl_lane_table_t>(lanes, "lanes"), as_struct<ttrl_params_t>(params, "params"),
                        as_struct<ttrl_reset_cfg_t>(cfg, "cfg"), reinterpret_cast<const uint64_t*>(pcg.data_ptr()),
                        stream_of(state[0])),
     "ttrl_reset_highway");
}

at::Tensor entropy_words(const at::Tensor& entropy, const ttrl_state_t& s, const at::Tensor& like) {
  TORCH_CHECK(entropy.dim() == 2 && entropy.size(0) == s.n_envs && entropy.scalar_type() == at::kInt,
              "ttrl: entropy must be an int32 [n_envs, n_words] tensor of uint32 words");
  TORCH_CHECK(entropy.device() == like.device(), "ttrl: entropy must live on the state's device");
  return entropy.contiguous();
}

void reset_highway_seeded_(at::TensorList state, const at::Tensor& lanes, const at::Tensor& params,
                           const at::Tensor& cfg, const at::Tensor& entropy, const c10::optional<at::Tensor>& mask) {
  check_hip(state[0]);
  ttrl_state_t s = state_of(state);
  at::Tensor w = entropy_words(entropy, s, state[0]);
  at::Tensor m = dev_u8(mask, s.n_envs, state[0], "mask");
  ok(ttrl_reset_highway_seeded(&s, as_struct<ttrl_lane_table_t>(lanes, "lanes"),
                               as_struct<ttrl_params_t>(params, "params"), as_struct<ttrl_reset_cfg_t>(cfg, "cfg"),
                               reinterpret_cast<const uint32_t*>(w.data_ptr()), static_cast<int32_t>(w.size(1)),
                               static_cast<const uint8_t*>(ptr(m)), stream_of(state[0])),
     "ttrl_reset_highway_seeded");
}

void check_time(const at::Tensor& time, const ttrl_state_t& s, const at::Tensor& like);

// VecHighwayEnv.step's auto-reset: done = terminated | truncated (returned), the done envs' episode
// word bumped, their scenes regenerated from the bumped entropy and their time zeroed.
at::Tensor auto_reset_highway_(at::TensorList state, const at::Tensor& lanes, const at::Tensor& params,
                               const at::Tensor& cfg, const at::Tensor& entropy, int64_t episode_word,
                               const at::Tensor& terminated, const at::Tensor& truncated, const at::Tensor& time) {
  check_hip(state[0]);
  ttrl_state_t s = state_of(state);
  TORCH_CHECK(entropy.dim() == 2 && entropy.size(0) == s.n_envs && entropy.scalar_type() == at::kInt &&
                  entropy.is_contiguous() && entropy.device() == state[0].device(),
              "ttrl: entropy must be a contiguous int32 [n_envs, n_words] tensor on the state's device");
  for (const at::Tensor* t : {&terminated, &truncated})
    TORCH_CHECK(t->device() == state[0].device() && t->numel() == s.n_envs && t->is_contiguous() &&
                    (t->scalar_type() == at::kBool || t->scalar_type() == at::kByte),
                "ttrl: terminated / truncated must be contiguous bool [n_envs] tensors on the state's device");
  check_time(time, s, state[0]);
  at::Tensor done = at::empty({s.n_envs}, opts(state[0], at::kBool));
  ok(ttrl_auto_reset_highway(&s, as_struct<ttrl_lane_table_t>(lanes, "lanes"), as_struct<ttrl_params_t>(params, "params"),
                             as_struct<ttrl_reset_cfg_t>(cfg, "cfg"), reinterpret_cast<uint32_t*>(entropy.data_ptr()),
                             static_cast<int32_t>(entropy.size(1)), static_cast<int32_t>(episode_word),
                             static_cast<const uint8_t*>(terminated.data_ptr()),
                             static_cast<const uint8_t*>(truncated.data_ptr()), time.data_ptr<double>(),
                             static_cast<uint8_t*>(done.data_ptr()), stream_of(state[0])),
     "ttrl_auto_reset_highway");
  return done;
}

void ix_reset_(at::TensorList state, const at::Tensor& lanes, const at::Tensor& params, const at::Tensor& cfg,
               const at::Tensor& entropy, const c10::optional<at::Tensor>& mask) {
  check_hip(state[0]);
  ttrl_state_t s = state_of(state);
  at::Tensor w = entropy_words(entropy, s, state[0]);
  at::Tensor m = dev_u8(mask, s.n_envs, state[0], "mask");
  ok(ttrl_ix_reset(&s, as_struct<ttrl_lane_table_t>(lanes, "lanes"), as_struct<ttrl_params_t>(params, "params"),
                   as_struct<ttrl_ix_cfg_t>(cfg, "cfg"), reinterpret_cast<const uint32_t*>(w.data_ptr()),
                   static_cast<int32_t>(w.size(1)), static_cast<const uint8_t*>(ptr(m)), stream_of(state[0])),
     "ttrl_ix_reset");
}

// ttrl_ix_reset in parts (bits 1 begin, 2 warm-up frames, 4 finish), each over its own mask.
void ix_reset_parts_(at::TensorList state, const at::Tensor& lanes, const at::Tensor& params, const at::Tensor& cfg,
                     int64_t parts, const c10::optional<at::Tensor>& entropy,
                     const c10::optional<at::Tensor>& begin_mask, const c10::optional<at::Tensor>& warm_mask,
                     int64_t warm_frames, const c10::optional<at::Tensor>& finish_mask) {
  check_hip(state[0]);
  ttrl_state_t s = state_of(state);
  TORCH_CHECK(parts >= 0 && parts <= 7 && warm_frames >= 0, "ttrl: parts must be a mask of 1 | 2 | 4");
  at::Tensor w;
  if (parts & TTRL_IX_BEGIN) {
    TORCH_CHECK(entropy && entropy->defined(), "ttrl: the begin part needs the entropy words");
    w = entropy_words(*entropy, s, state[0]);
  }
  at::Tensor bm = dev_u8(begin_mask, s.n_envs, state[0], "begin_mask");
  at::Tensor wm = dev_u8(warm_mask, s.n_envs, state[0], "warm_mask");
  at::Tensor fm = dev_u8(finish_mask, s.n_envs, state[0], "finish_mask");
  ok(ttrl_ix_reset_parts(&s, as_struct<ttrl_lane_table_t>(lanes, "lanes"), as_struct<ttrl_params_t>(params, "params"),
                         as_struct<ttrl_ix_cfg_t>(cfg, "cfg"), static_cast<int32_t>(parts),
                         w.defined() ? reinterpret_cast<const uint32_t*>(w.data_ptr()) : nullptr,
                         w.defined() ? static_cast<int32_t>(w.size(1)) : 0, static_cast<const uint8_t*>(ptr(bm)),
                         static_cast<const uint8_t*>(ptr(wm)), static_cast<int32_t>(warm_frames),
                         static_cast<const uint8_t*>(ptr(fm)), stream_of(state[0])),
     "ttrl_ix_reset_parts");
}

void ix_clear_spawn_(at::TensorList state, const at::Tensor& lanes, const at::Tensor& params, const at::Tensor& cfg,
                     const c10::optional<at::Tensor>& mask) {
  check_hip(state[0]);
  ttrl_state_t s = state_of(state);
  at::Tensor m = dev_u8(mask, s.n_envs, state[0], "mask");
  ok(ttrl_ix_clear_spawn(&s, as_struct<ttrl_lane_table_t>(lanes, "lanes"), as_struct<ttrl_params_t>(params, "params"),
                         as_struct<ttrl_ix_cfg_t>(cfg, "cfg"), static_cast<const uint8_t*>(ptr(m)),
                         stream_of(state[0])),
     "ttrl_ix_clear_spawn");
}

// VecIntersectionEnv.step after env_step_: clear / spawn for the envs that go on, the auto-reset of
// the finished ones from the spare scenes (2E rows) and their first observation.  Returns
// (done [E] bool, spare_mask [2E] uint8: the spare rows to reset again, obs [E, V, F], ids).
// live_count (optional int64 scalar): += the vehicles present after the tail.
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> ix_step_tail_(
    at::TensorList state, const at::Tensor& lanes, const at::Tensor& params, const at::Tensor& cfg,
    at::TensorList spare, const at::Tensor& terminated, const at::Tensor& truncated, const at::Tensor& spare_parity,
    const at::Tensor& entropy, const at::Tensor& spare_entropy, const at::Tensor& time,
    const c10::optional<at::Tensor>& kin_cfg, const c10::optional<at::Tensor>& obs,
    const c10::optional<at::Tensor>& ids, const c10::optional<at::Tensor>& live_count,
    const c10::optional<at::Tensor>& order) {
  check_hip(state[0]);
  ttrl_state_t s = state_of(state), sp = state_of(spare);
  const auto& x = state[0];
  const int64_t K = s.n_envs > 0 ? sp.n_envs / s.n_envs : 0;  // spare slots per env
  TORCH_CHECK(spare[0].device() == x.device() && K >= 2 && K <= 16 && sp.n_envs == K * s.n_envs &&
                  sp.n_veh == s.n_veh &&
                  sp.dtype == s.dtype,
              "ttrl: spare must be a state of K * n_envs rows (K in [2, 16]) of the same width and dtype on the "
              "state's device");
  for (const at::Tensor* t : {&terminated, &truncated})
    TORCH_CHECK(t->device() == x.device() && t->numel() == s.n_envs && t->is_contiguous() &&
                    (t->scalar_type() == at::kBool || t->scalar_type() == at::kByte),
                "ttrl: terminated / truncated must be contiguous bool [n_envs] tensors on the state's device");
  TORCH_CHECK(spare_parity.device() == x.device() && spare_parity.scalar_type() == at::kByte &&
                  spare_parity.is_contiguous() && spare_parity.numel() == s.n_envs,
              "ttrl: spare_parity must be a contiguous uint8 [n_envs] tensor on the state's device");
  TORCH_CHECK(entropy.dim() == 2 && entropy.size(0) == s.n_envs && entropy.scalar_type() == at::kInt &&
                  entropy.is_contiguous() && entropy.device() == x.device(),
              "ttrl: entropy must be a contiguous int32 [n_envs, n_words] tensor on the state's device");
  TORCH_CHECK(spare_entropy.dim() == 2 && spare_entropy.size(0) == sp.n_envs &&
                  spare_entropy.size(1) == entropy.size(1) && spare_entropy.scalar_type() == at::kInt &&
                  spare_entropy.is_contiguous() && spare_entropy.device() == x.device(),
              "ttrl: spare_entropy must be a contiguous int32 [K * n_envs, n_words] tensor on the state's device");
  check_time(time, s, x);
  const ttrl_kin_cfg_t* kc = kin_cfg && kin_cfg->defined() ? as_struct<ttrl_kin_cfg_t>(*kin_cfg, "kin_cfg") : nullptr;
  at::Tensor obs_out, ids_out, oin, iin;
  if (kc) {
    TORCH_CHECK(obs && obs->defined() && ids && ids->defined(), "ttrl: a kin_cfg needs the step's obs and ids");
    std::tie(obs_out, ids_out) = kin_outputs(x, kc);
    oin = obs->contiguous();
    iin = ids->contiguous();
    TORCH_CHECK(oin.device() == x.device() && oin.scalar_type() == at::kFloat && oin.sizes() == obs_out.sizes(),
                "ttrl: obs must be the step's float32 [E, V, F] observation");
    TORCH_CHECK(iin.device() == x.device() && iin.scalar_type() == at::kInt && iin.sizes() == ids_out.sizes(),
                "ttrl: ids must be the step's int32 [E, V-1] observed ids");
  } else {
    obs_out = at::empty({0}, opts(x, at::kFloat));
    ids_out = at::empty({0}, opts(x, at::kInt));
  }
  const bool lc = live_count && live_count->defined();
  if (lc)
    TORCH_CHECK(live_count->device() == x.device() && live_count->scalar_type() == at::kLong &&
                    live_count->numel() == 1,
                "ttrl: live_count must be an int64 scalar on the state's device");
  const bool od = order && order->defined();
  if (od)
    TORCH_CHECK(order->device() == x.device() && order->scalar_type() == at::kInt && order->is_contiguous() &&
                    order->numel() == 2 * int64_t(s.n_envs),
                "ttrl: order must be a contiguous int32 [2 * n_envs] tensor on the state's device");
  at::Tensor done = at::empty({s.n_envs}, opts(x, at::kBool));
  at::Tensor smask = at::empty({sp.n_envs}, opts(x, at::kByte));
  ok(ttrl_ix_step_tail(&s, as_struct<ttrl_lane_table_t>(lanes, "lanes"), as_struct<ttrl_params_t>(params, "params"),
                       as_struct<ttrl_ix_cfg_t>(cfg, "cfg"), &sp, static_cast<const uint8_t*>(terminated.data_ptr()),
                       static_cast<const uint8_t*>(truncated.data_ptr()),
                       static_cast<uint8_t*>(spare_parity.data_ptr()), reinterpret_cast<uint32_t*>(entropy.data_ptr()),
                       reinterpret_cast<uint32_t*>(spare_entropy.data_ptr()), static_cast<int32_t>(entropy.size(1)),
                       time.data_ptr<double>(), static_cast<uint8_t*>(done.data_ptr()),
                       static_cast<uint8_t*>(smask.data_ptr()), kc, kc ? oin.data_ptr<float>() : nullptr,
                       kc ? obs_out.data_ptr<float>() : nullptr, kc ? iin.data_ptr<int32_t>() : nullptr,
                       kc ? ids_out.data_ptr<int32_t>() : nullptr, lc ? live_count->data_ptr<int64_t>() : nullptr,
                       od ? order->data_ptr<int32_t>() : nullptr, stream_of(x)),
     "ttrl_ix_step_tail");
  return {done, smask, obs_out, ids_out};
}

// VecIntersectionEnv.step with the auto-reset from spare scenes, in one launch (ttrl_ix_env_step):
// env_step_'s eight outputs, then done [E] bool, spare_mask [K * E] uint8 and the next observation
// obs_next / ids_next -- ix_step_tail_'s outputs -- with the same spare / parity / entropy / time /
// live_count / order arguments as env_step_ followed by ix_step_tail_.
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor,
           at::Tensor, at::Tensor, at::Tensor>
ix_env_step_(at::TensorList state, const at::Tensor& lanes, const at::Tensor& params, const at::Tensor& cfg,
             const c10::optional<at::Tensor>& actions, int64_t frames, double dt, const at::Tensor& kin_cfg,
             const at::Tensor& reward_cfg, const at::Tensor& time, double time_inc, at::TensorList spare,
             const at::Tensor& spare_parity, const at::Tensor& entropy, const at::Tensor& spare_entropy,
             const c10::optional<at::Tensor>& order, at::OptionalIntArrayRef action_lut,
             const c10::optional<at::Tensor>& live_count) {
  check_hip(state[0]);
  ttrl_state_t s = state_of(state), sp = state_of(spare);
  const auto& x = state[0];
  const auto* kc = as_struct<ttrl_kin_cfg_t>(kin_cfg, "kin_cfg");
  check_time(time, s, x);
  const int64_t K = s.n_envs > 0 ? sp.n_envs / s.n_envs : 0;
  TORCH_CHECK(spare[0].device() == x.device() && K >= 2 && K <= 16 && sp.n_envs == K * s.n_envs &&
                  sp.n_veh == s.n_veh && sp.dtype == s.dtype,
              "ttrl: spare must be a state of K * n_envs rows (K in [2, 16]) of the same width and dtype on the "
              "state's device");
  TORCH_CHECK(spare_parity.device() == x.device() && spare_parity.scalar_type() == at::kByte &&
                  spare_parity.is_contiguous() && spare_parity.numel() == s.n_envs,
              "ttrl: spare_parity must be a contiguous uint8 [n_envs] tensor on the state's device");
  TORCH_CHECK(entropy.dim() == 2 && entropy.size(0) == s.n_envs && entropy.scalar_type() == at::kInt &&
                  entropy.is_contiguous() && entropy.device() == x.device(),
              "ttrl: entropy must be a contiguous int32 [n_envs, n_words] tensor on the state's device");
  TORCH_CHECK(spare_entropy.dim() == 2 && spare_entropy.size(0) == sp.n_envs &&
                  spare_entropy.size(1) == entropy.size(1) && spare_entropy.scalar_type() == at::kInt &&
                  spare_entropy.is_contiguous() && spare_entropy.device() == x.device(),
              "ttrl: spare_entropy must be a contiguous int32 [K * n_envs, n_words] tensor on the state's device");
  at::Tensor a = dev_i32(actions, s.n_envs, x, "actions");
  const bool od = order && order->defined();
  if (od)
    TORCH_CHECK(order->device() == x.device() && order->scalar_type() == at::kInt && order->is_contiguous() &&
                    order->numel() == 2 * int64_t(s.n_envs),
                "ttrl: order must be a contiguous int32 [2 * n_envs] tensor on the state's device");
  const bool lc = live_count && live_count->defined();
  if (lc)
    TORCH_CHECK(live_count->device() == x.device() && live_count->scalar_type() == at::kLong &&
                    live_count->numel() == 1,
                "ttrl: live_count must be an int64 scalar on the state's device");
  std::vector<int32_t> lut;
  if (action_lut.has_value())
    for (int64_t c : *action_lut) lut.push_back(static_cast<int32_t>(c));
  auto [obs, ids, rew, term, trunc, comp, speed, crashed] = env_step_outputs(x, kc);
  auto [obs2, ids2] = kin_outputs(x, kc);
  at::Tensor done = at::empty({s.n_envs}, opts(x, at::kBool));
  at::Tensor smask = at::empty({sp.n_envs}, opts(x, at::kByte));
  ok(ttrl_ix_env_step(&s, as_struct<ttrl_lane_table_t>(lanes, "lanes"), as_struct<ttrl_params_t>(params, "params"),
                      as_struct<ttrl_ix_cfg_t>(cfg, "cfg"), static_cast<const int32_t*>(ptr(a)),
                      static_cast<int32_t>(frames), dt, kc, obs.data_ptr<float>(), ids.data_ptr<int32_t>(),
                      obs2.data_ptr<float>(), ids2.data_ptr<int32_t>(),
                      as_struct<ttrl_reward_cfg_t>(reward_cfg, "reward_cfg"), time.data_ptr<double>(), time_inc,
                      rew.data_ptr<float>(), static_cast<uint8_t*>(term.data_ptr()),
                      static_cast<uint8_t*>(trunc.data_ptr()), comp.data_ptr<float>(), speed.data_ptr(),
                      static_cast<uint8_t*>(crashed.data_ptr()), &sp, static_cast<uint8_t*>(spare_parity.data_ptr()),
                      reinterpret_cast<uint32_t*>(entropy.data_ptr()),
                      reinterpret_cast<uint32_t*>(spare_entropy.data_ptr()), static_cast<int32_t>(entropy.size(1)),
                      static_cast<uint8_t*>(done.data_ptr()), static_cast<uint8_t*>(smask.data_ptr()),
                      od ? order->data_ptr<int32_t>() : nullptr, lut.empty() ? nullptr : lut.data(),
                      static_cast<int32_t>(lut.size()), lc ? live_count->data_ptr<int64_t>() : nullptr, stream_of(x)),
     "ttrl_ix_env_step");
  return {obs, ids, rew, term, trunc, comp, speed, crashed, done, smask, obs2, ids2};
}

void copy_envs_(at::TensorList dst, at::TensorList src, const at::Tensor& mask) {
  check_hip(dst[0]);
  ttrl_state_t d = state_of(dst), s = state_of(src);
  TORCH_CHECK(d.n_envs == s.n_envs && d.n_veh == s.n_veh && d.dtype == s.dtype && dst[0].device() == src[0].device(),
              "ttrl: copy_envs needs two states of one shape, dtype and device");
  at::Tensor m = dev_u8(mask, d.n_envs, dst[0], "mask");
  ok(ttrl_copy_envs(&d, &s, static_cast<const uint8_t*>(ptr(m)), stream_of(dst[0])), "ttrl_copy_envs");
}

// ------------------------------------------------------------------------------------ rewards
void check_time(const at::Tensor& time, const ttrl_state_t& s, const at::Tensor& like) {
  TORCH_CHECK(time.device() == like.device() && time.scalar_type() == at::kDouble && time.is_contiguous() &&
                  time.numel() == s.n_envs,
              "ttrl: time must be a contiguous float64 [n_envs] tensor on the state's device");
}

std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> rewards_ex(at::TensorList state, const at::Tensor& lanes,
                                                                      const at::Tensor& cfg, const at::Tensor& time) {
  check_hip(state[0]);
  ttrl_state_t s = state_of(state);
  check_time(time, s, state[0]);
  const auto& x = state[0];
  at::Tensor rew = at::empty({s.n_envs}, opts(x, at::kFloat)), term = at::empty({s.n_envs}, opts(x, at::kBool)),
             trunc = at::empty({s.n_envs}, opts(x, at::kBool)), comp = at::empty({s.n_envs, 4}, opts(x, at::kFloat));
  ok(ttrl_rewards_ex(&s, as_struct<ttrl_lane_table_t>(lanes, "lanes"), as_struct<ttrl_reward_cfg_t>(cfg, "cfg"),
                     time.data_ptr<double>(), rew.data_ptr<float>(), static_cast<uint8_t*>(term.data_ptr()),
                     static_cast<uint8_t*>(trunc.data_ptr()), comp.data_ptr<float>(), stream_of(x)),
     "ttrl_rewards_ex");
  return {rew, term, trunc, comp};
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> rewards(at::TensorList state, const at::Tensor& lanes,
                                                       const at::Tensor& cfg, const at::Tensor& time) {
  check_hip(state[0]);
  ttrl_state_t s = state_of(state);
  check_time(time, s, state[0]);
  const auto& x = state[0];
  at::Tensor rew = at::empty({s.n_envs}, opts(x, at::kFloat)), term = at::empty({s.n_envs}, opts(x, at::kBool)),
             trunc = at::empty({s.n_envs}, opts(x, at::kBool));
  ok(ttrl_rewards(&s, as_struct<ttrl_lane_table_t>(lanes, "lanes"), as_struct<ttrl_reward_cfg_t>(cfg, "cfg"),
                  time.data_ptr<double>(), rew.data_ptr<float>(), static_cast<uint8_t*>(term.data_ptr()),
                  static_cast<uint8_t*>(trunc.data_ptr()), stream_of(x)),
     "ttrl_rewards");
  return {rew, term, trunc};
}

std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor> rewards_step_(
    at::TensorList state, const at::Tensor& lanes, const at::Tensor& cfg, const at::Tensor& time, double time_inc) {
  check_hip(state[0]);
  ttrl_state_t s = state_of(state);
  check_time(time, s, state[0]);
  const auto& x = state[0];
  at::Tensor rew = at::empty({s.n_envs}, opts(x, at::kFloat)), term = at::empty({s.n_envs}, opts(x, at::kBool)),
             trunc = at::empty({s.n_envs}, opts(x, at::kBool)), comp = at::empty({s.n_envs, 4}, opts(x, at::kFloat)),
             speed = at::empty({s.n_envs}, opts(x, x.scalar_type())), crashed = at::empty({s.n_envs}, opts(x, at::kBool));
  ok(ttrl_rewards_step(&s, as_struct<ttrl_lane_table_t>(lanes, "lanes"), as_struct<ttrl_reward_cfg_t>(cfg, "cfg"),
                       time.data_ptr<double>(), time_inc, rew.data_ptr<float>(), static_cast<uint8_t*>(term.data_ptr()),
                       static_cast<uint8_t*>(trunc.data_ptr()), comp.data_ptr<float>(), speed.data_ptr(),
                       static_cast<uint8_t*>(crashed.data_ptr()), stream_of(x)),
     "ttrl_rewards_step");
  return {rew, term, trunc, comp, speed, crashed};
}

// ------------------------------------------------------------------------------------ policy
at::Tensor ego_attention_q(const at::Tensor& obs, const at::Tensor& weights, int64_t heads, int64_t n_actions) {
  check_hip(obs);
  TORCH_CHECK(obs.dim() == 3 && obs.scalar_type() == at::kFloat, "ttrl: obs must be float32 [B, entities, features]");
  TORCH_CHECK(weights.device() == obs.device() && weights.scalar_type() == at::kFloat && weights.is_contiguous(),
              "ttrl: weights must be a contiguous float32 tensor on the obs device (packed layout)");
  at::Tensor x = obs.contiguous();
  const int32_t B = x.size(0), NE = x.size(1), F = x.size(2);
  int64_t n_scratch = 0;
  const int64_t n_w = ttrl_ego_attention_sizes(F, static_cast<int32_t>(n_actions), B, NE, &n_scratch);
  TORCH_CHECK(n_w > 0 && weights.numel() == n_w, "ttrl: packed weights need ", n_w, " floats, got ", weights.numel());
  at::Tensor scratch = at::empty({std::max<int64_t>(n_scratch, 1)}, opts(x, at::kFloat));
  at::Tensor q = at::empty({B, n_actions}, opts(x, at::kFloat));
  ok(ttrl_ego_attention_q(x.data_ptr<float>(), B, NE, F, static_cast<int32_t>(heads), weights.data_ptr<float>(),
                          static_cast<int32_t>(n_actions), scratch.data_ptr<float>(), q.data_ptr<float>(), stream_of(x)),
     "ttrl_ego_attention_q");
  return q;
}

// EgoAttention Q-values and the epsilon-greedy actions in one launch (ttrl_ego_attention_act):
// returns (actions [B] int64, or int32 with int32_actions -- the env's action index type, so the
// step takes them without a cast launch; q [B, A] float32).  epsilon_dev / step_dev: optional device
// scalars (float32 / int64) that override epsilon / step inside the kernel (captured graphs).
std::tuple<at::Tensor, at::Tensor> ego_attention_act(const at::Tensor& obs, const at::Tensor& weights, int64_t heads,
                                                     int64_t n_actions, double epsilon, int64_t seed, int64_t step,
                                                     const c10::optional<at::Tensor>& epsilon_dev,
                                                     const c10::optional<at::Tensor>& step_dev,
                                                     bool int32_actions, int64_t env_offset) {
  check_hip(obs);
  TORCH_CHECK(obs.dim() == 3 && obs.scalar_type() == at::kFloat, "ttrl: obs must be float32 [B, entities, features]");
  TORCH_CHECK(weights.device() == obs.device() && weights.scalar_type() == at::kFloat && weights.is_contiguous(),
              "ttrl: weights must be a contiguous float32 tensor on the obs device (packed layout)");
  TORCH_CHECK(epsilon >= 0.0 && epsilon <= 1.0, "ttrl: epsilon must lie in [0, 1]");
  TORCH_CHECK(env_offset >= 0, "ttrl: env_offset must be non-negative");
  const bool ed = epsilon_dev && epsilon_dev->defined(), sd = step_dev && step_dev->defined();
  if (ed)
    TORCH_CHECK(epsilon_dev->device() == obs.device() && epsilon_dev->scalar_type() == at::kFloat &&
                    epsilon_dev->numel() == 1,
                "ttrl: epsilon_dev must be a float32 scalar on the obs device");
  if (sd)
    TORCH_CHECK(step_dev->device() == obs.device() && step_dev->scalar_type() == at::kLong && step_dev->numel() == 1,
                "ttrl: step_dev must be an int64 scalar on the obs device");
  at::Tensor x = obs.contiguous();
  const int32_t B = x.size(0), NE = x.size(1), F = x.size(2);
  int64_t n_scratch = 0;
  const int64_t n_w = ttrl_ego_attention_sizes(F, static_cast<int32_t>(n_actions), B, NE, &n_scratch);
  TORCH_CHECK(n_w > 0 && weights.numel() == n_w, "ttrl: packed weights need ", n_w, " floats, got ", weights.numel());
  at::Tensor q = at::empty({B, n_actions}, opts(x, at::kFloat));
  at::Tensor act = at::empty({B}, opts(x, int32_actions ? at::kInt : at::kLong));
  ok(ttrl_ego_attention_act(x.data_ptr<float>(), B, NE, F, static_cast<int32_t>(heads), weights.data_ptr<float>(),
                            static_cast<int32_t>(n_actions), static_cast<float>(epsilon),
                            ed ? epsilon_dev->data_ptr<float>() : nullptr, static_cast<uint64_t>(seed), step,
                            sd ? step_dev->data_ptr<int64_t>() : nullptr, env_offset, q.data_ptr<float>(),
                            int32_actions ? nullptr : act.data_ptr<int64_t>(),
                            int32_actions ? act.data_ptr<int32_t>() : nullptr, stream_of(x)),
     "ttrl_ego_attention_act");
  return {act, q};
}

// ------------------------------------------------------------------------------------ Meta kernels
const at::Tensor& meta_x(at::TensorList ts) {
  TORCH_CHECK(ts.size() == kFields, "ttrl: state must hold ", kFields, " tensors in _abi.ALL_FIELDS order, got ",
              ts.size());
  TORCH_CHECK(ts[0].dim() == 2, "ttrl: state tensors are [n_envs, n_veh]");
  return ts[0];
}

void meta_none_sim(at::TensorList, const at::Tensor&, const at::Tensor&, const c10::optional<at::Tensor>&, int64_t,
                   double) {}
void meta_none_act(at::TensorList, const at::Tensor&, const at::Tensor&) {}
void meta_none_step(at::TensorList, const at::Tensor&, const at::Tensor&, double) {}
void meta_none_meta(at::TensorList, const at::Tensor&, const at::Tensor&, const at::Tensor&) {}

std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor>
meta_env_step(at::TensorList state, const at::Tensor&, const at::Tensor&, const c10::optional<at::Tensor>&, int64_t,
              double, const c10::optional<at::Tensor>& kin_cfg, const at::Tensor&, const at::Tensor&, double,
              const c10::optional<at::Tensor>&, at::OptionalIntArrayRef, const c10::optional<at::Tensor>& grid_cfg) {
  const ttrl_kin_cfg_t* kc = kin_cfg && kin_cfg->defined() ? as_struct<ttrl_kin_cfg_t>(*kin_cfg, "kin_cfg") : nullptr;
  const ttrl_grid_cfg_t* gc =
      grid_cfg && grid_cfg->defined() ? as_struct<ttrl_grid_cfg_t>(*grid_cfg, "grid_cfg") : nullptr;
  return env_step_outputs(meta_x(state), kc, gc);
}

std::tuple<at::Tensor, at::Tensor> meta_neighbours(at::TensorList state, const at::Tensor& lanes,
                                                   const c10::optional<at::Tensor>&) {
  as_struct<ttrl_lane_table_t>(lanes, "lanes");
  at::Tensor f = at::empty({meta_x(state).size(0), meta_x(state).size(1)}, opts(meta_x(state), at::kInt));
  return {f, at::empty_like(f)};
}

std::tuple<at::Tensor, at::Tensor> meta_kin(at::TensorList state, const at::Tensor&, const at::Tensor&,
                                            const at::Tensor& cfg) {
  return kin_outputs(meta_x(state), as_struct<ttrl_kin_cfg_t>(cfg, "cfg"));
}

void meta_kin_masked(at::TensorList, const at::Tensor&, const at::Tensor&, const at::Tensor&, const at::Tensor&,
                     const at::Tensor&, const at::Tensor&) {}

at::Tensor meta_grid(at::TensorList state, const at::Tensor&, const at::Tensor&, const at::Tensor& cfg) {
  const auto* c = as_struct<ttrl_grid_cfg_t>(cfg, "cfg");
  return at::empty({meta_x(state).size(0), c->n_features, c->shape_x, c->shape_y}, opts(meta_x(state), at::kFloat));
}

at::Tensor meta_ttc(at::TensorList state, const at::Tensor& lanes, const at::Tensor& params, const at::Tensor& cfg) {
  return at::empty(ttc_shape(meta_x(state).size(0), as_struct<ttrl_lane_table_t>(lanes, "lanes"),
                             as_struct<ttrl_params_t>(params, "params"), as_struct<ttrl_ttc_cfg_t>(cfg, "cfg")),
                   opts(meta_x(state), at::kFloat));
}

at::Tensor meta_lidar(at::TensorList state, const at::Tensor&, const at::Tensor&, const at::Tensor& cfg) {
  return at::empty({meta_x(state).size(0), as_struct<ttrl_lidar_cfg_t>(cfg, "cfg")->cells, 2}, opts(meta_x(state), at::kFloat));
}

void meta_reset(at::TensorList, const at::Tensor&, const at::Tensor&, const at::Tensor&, const at::Tensor&) {}
void meta_reset_seeded(at::TensorList, const at::Tensor&, const at::Tensor&, const at::Tensor&, const at::Tensor&,
                       const c10::optional<at::Tensor>&) {}
void meta_ix_reset_parts(at::TensorList, const at::Tensor&, const at::Tensor&, const at::Tensor&, int64_t,
                         const c10::optional<at::Tensor>&, const c10::optional<at::Tensor>&,
                         const c10::optional<at::Tensor>&, int64_t, const c10::optional<at::Tensor>&) {}
void meta_clear_spawn(at::TensorList, const at::Tensor&, const at::Tensor&, const at::Tensor&,
                      const c10::optional<at::Tensor>&) {}
void meta_copy_envs(at::TensorList, at::TensorList, const at::Tensor&) {}
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> meta_ix_step_tail(
    at::TensorList state, const at::Tensor&, const at::Tensor&, const at::Tensor&, at::TensorList, const at::Tensor&,
    const at::Tensor&, const at::Tensor&, const at::Tensor&, const at::Tensor&, const at::Tensor&,
    const c10::optional<at::Tensor>& kin_cfg, const c10::optional<at::Tensor>&, const c10::optional<at::Tensor>&,
    const c10::optional<at::Tensor>&, const c10::optional<at::Tensor>&) {
  const auto& x = meta_x(state);
  const int64_t E = x.size(0);
  at::Tensor o = at::empty({0}, opts(x, at::kFloat)), i = at::empty({0}, opts(x, at::kInt));
  if (kin_cfg && kin_cfg->defined()) std::tie(o, i) = kin_outputs(x, as_struct<ttrl_kin_cfg_t>(*kin_cfg, "kin_cfg"));
  return {at::empty({E}, opts(x, at::kBool)), at::empty({2 * E}, opts(x, at::kByte)), o, i};
}
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor,
           at::Tensor, at::Tensor, at::Tensor>
meta_ix_env_step(at::TensorList state, const at::Tensor&, const at::Tensor&, const at::Tensor&,
                 const c10::optional<at::Tensor>&, int64_t, double, const at::Tensor& kin_cfg, const at::Tensor&,
                 const at::Tensor&, double, at::TensorList spare, const at::Tensor&, const at::Tensor&,
                 const at::Tensor&, const c10::optional<at::Tensor>&, at::OptionalIntArrayRef,
                 const c10::optional<at::Tensor>&) {
  const auto& x = meta_x(state);
  const auto* kc = as_struct<ttrl_kin_cfg_t>(kin_cfg, "kin_cfg");
  auto [obs, ids, rew, term, trunc, comp, speed, crashed] = env_step_outputs(x, kc);
  auto [obs2, ids2] = kin_outputs(x, kc);
  return {obs, ids, rew, term, trunc, comp, speed, crashed, at::empty({x.size(0)}, opts(x, at::kBool)),
          at::empty({meta_x(spare).size(0)}, opts(x, at::kByte)), obs2, ids2};
}
at::Tensor meta_auto_reset(at::TensorList state, const at::Tensor&, const at::Tensor&, const at::Tensor&,
                           const at::Tensor&, int64_t, const at::Tensor&, const at::Tensor&, const at::Tensor&) {
  return at::empty({meta_x(state).size(0)}, opts(meta_x(state), at::kBool));
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> meta_rewards(at::TensorList state, const at::Tensor&,
                                                            const at::Tensor&, const at::Tensor&) {
  const int64_t E = meta_x(state).size(0);
  return {at::empty({E}, opts(meta_x(state), at::kFloat)), at::empty({E}, opts(meta_x(state), at::kBool)),
          at::empty({E}, opts(meta_x(state), at::kBool))};
}

std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> meta_rewards_ex(at::TensorList state, const at::Tensor&,
                                                                           const at::Tensor&, const at::Tensor&) {
  const int64_t E = meta_x(state).size(0);
  return {at::empty({E}, opts(meta_x(state), at::kFloat)), at::empty({E}, opts(meta_x(state), at::kBool)),
          at::empty({E}, opts(meta_x(state), at::kBool)), at::empty({E, 4}, opts(meta_x(state), at::kFloat))};
}

std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor> meta_rewards_step(
    at::TensorList state, const at::Tensor&, const at::Tensor&, const at::Tensor&, double) {
  const auto& x = meta_x(state);
  const int64_t E = x.size(0);
  return {at::empty({E}, opts(x, at::kFloat)), at::empty({E}, opts(x, at::kBool)), at::empty({E}, opts(x, at::kBool)),
          at::empty({E, 4}, opts(x, at::kFloat)), at::empty({E}, opts(x, x.scalar_type())),
          at::empty({E}, opts(x, at::kBool))};
}

at::Tensor meta_ego_attention(const at::Tensor& obs, const at::Tensor&, int64_t, int64_t n_actions) {
  return at::empty({obs.size(0), n_actions}, opts(obs, at::kFloat));
}
std::tuple<at::Tensor, at::Tensor> meta_ego_attention_act(const at::Tensor& obs, const at::Tensor&, int64_t,
                                                          int64_t n_actions, double, int64_t, int64_t,
                                                          const c10::optional<at::Tensor>&,
                                                          const c10::optional<at::Tensor>&, bool int32_actions,
                                                          int64_t) {
  return {at::empty({obs.size(0)}, opts(obs, int32_actions ? at::kInt : at::kLong)),
          at::empty({obs.size(0), n_actions}, opts(obs, at::kFloat))};
}

}  // namespace

TORCH_LIBRARY(ttrl, m) {
  m.def("simulate_(Tensor(a!)[] state, Tensor lanes, Tensor params, Tensor? actions, int frames, float dt) -> ()");
  m.def("road_act_(Tensor(a!)[] state, Tensor lanes, Tensor params) -> ()");
  m.def("road_step_(Tensor(a!)[] state, Tensor lanes, Tensor params, float dt) -> ()");
  m.def("meta_action_(Tensor(a!)[] state, Tensor lanes, Tensor params, Tensor actions) -> ()");
  m.def("env_step_(Tensor(a!)[] state, Tensor lanes, Tensor params, Tensor? actions, int frames, float dt, "
        "Tensor? kin_cfg, Tensor reward_cfg, Tensor(b!) time, float time_inc, Tensor? order=None, "
        "int[]? action_lut=None, Tensor? grid_cfg=None) -> (Tensor obs, Tensor ids, "
        "Tensor reward, Tensor terminated, Tensor truncated, Tensor components, Tensor ego_speed, Tensor ego_crashed)");
  m.def("neighbours(Tensor[] state, Tensor lanes, Tensor? query_lane) -> (Tensor front, Tensor rear)");
  // the np_random-shuffled observation (order_shuffled 2) advances state.rng: the state is mutated
  m.def("kinematics_obs(Tensor(a!)[] state, Tensor lanes, Tensor params, Tensor cfg) -> (Tensor obs, Tensor ids)");
  m.def("kinematics_obs_masked_(Tensor(a!)[] state, Tensor lanes, Tensor params, Tensor cfg, Tensor mask, "
        "Tensor(b!) out, Tensor(c!) ids) -> ()");
  m.def("occupancy_grid(Tensor[] state, Tensor lanes, Tensor params, Tensor cfg) -> Tensor");
  m.def("observe_ttc(Tensor[] state, Tensor lanes, Tensor params, Tensor cfg) -> Tensor");
  m.def("observe_lidar(Tensor[] state, Tensor lanes, Tensor params, Tensor cfg) -> Tensor");
  m.def("reset_highway_(Tensor(a!)[] state, Tensor lanes, Tensor params, Tensor cfg, Tensor pcg) -> ()");
  m.def("reset_highway_seeded_(Tensor(a!)[] state, Tensor lanes, Tensor params, Tensor cfg, Tensor entropy, "
        "Tensor? mask) -> ()");
  m.def("auto_reset_highway_(Tensor(a!)[] state, Tensor lanes, Tensor params, Tensor cfg, Tensor(b!) entropy, "
        "int episode_word, Tensor terminated, Tensor truncated, Tensor(c!) time) -> Tensor done");
  m.def("ix_reset_(Tensor(a!)[] state, Tensor lanes, Tensor params, Tensor cfg, Tensor entropy, Tensor? mask) -> ()");
  m.def("ix_reset_parts_(Tensor(a!)[] state, Tensor lanes, Tensor params, Tensor cfg, int parts, Tensor? entropy, "
        "Tensor? begin_mask, Tensor? warm_mask, int warm_frames, Tensor? finish_mask) -> ()");
  m.def("ix_clear_spawn_(Tensor(a!)[] state, Tensor lanes, Tensor params, Tensor cfg, Tensor? mask) -> ()");
  m.def("copy_envs_(Tensor(a!)[] dst, Tensor[] src, Tensor mask) -> ()");
  m.def("ix_step_tail_(Tensor(a!)[] state, Tensor lanes, Tensor params, Tensor cfg, Tensor[] spare, "
        "Tensor terminated, Tensor truncated, Tensor(b!) spare_parity, Tensor(c!) entropy, Tensor(d!) spare_entropy, "
        "Tensor(e!) time, Tensor? kin_cfg, Tensor? obs, Tensor? ids, Tensor(f!)? live_count=None, "
        "Tensor(g!)? order=None) -> (Tensor done, Tensor spare_mask, Tensor obs, Tensor ids)");
  m.def("ix_env_step_(Tensor(a!)[] state, Tensor lanes, Tensor params, Tensor cfg, Tensor? actions, int frames, "
        "float dt, Tensor kin_cfg, Tensor reward_cfg, Tensor(b!) time, float time_inc, Tensor[] spare, "
        "Tensor(e!) spare_parity, Tensor(f!) entropy, Tensor(g!) spare_entropy, Tensor(c!)? order=None, "
        "int[]? action_lut=None, Tensor(d!)? live_count=None) -> (Tensor obs, Tensor ids, Tensor reward, "
        "Tensor terminated, Tensor truncated, Tensor components, Tensor ego_speed, Tensor ego_crashed, "
        "Tensor done, Tensor spare_mask, Tensor obs_next, Tensor ids_next)");
  m.def("rewards(Tensor[] state, Tensor lanes, Tensor cfg, Tensor time) -> (Tensor reward, Tensor terminated, "
        "Tensor truncated)");
  m.def("rewards_ex(Tensor[] state, Tensor lanes, Tensor cfg, Tensor time) -> (Tensor reward, Tensor terminated, "
        "Tensor truncated, Tensor components)");
  m.def("rewards_step_(Tensor[] state, Tensor lanes, Tensor cfg, Tensor(a!) time, float time_inc) -> (Tensor reward, "
        "Tensor terminated, Tensor truncated, Tensor components, Tensor ego_speed, Tensor ego_crashed)");
  m.def("ego_attention_q(Tensor obs, Tensor weights, int heads, int n_actions) -> Tensor");
  m.def("ego_attention_act(Tensor obs, Tensor weights, int heads, int n_actions, float epsilon, int seed, int step, "
        "Tensor? epsilon_dev=None, Tensor? step_dev=None, bool int32_actions=False, int env_offset=0) -> (Tensor, Tensor)");
}

TORCH_LIBRARY_IMPL(ttrl, CUDA, m) {  // the HIP device of ROCm PyTorch
  m.impl("simulate_", &simulate_);
  m.impl("road_act_", &road_act_);
  m.impl("road_step_", &road_step_);
  m.impl("meta_action_", &meta_action_);
  m.impl("env_step_", &env_step_);
  m.impl("neighbours", &neighbours);
  m.impl("kinematics_obs", &kinematics_obs);
  m.impl("kinematics_obs_masked_", &kinematics_obs_masked_);
  m.impl("occupancy_grid", &occupancy_grid);
  m.impl("observe_ttc", &observe_ttc);
  m.impl("observe_lidar", &observe_lidar);
  m.impl("reset_highway_", &reset_highway_);
  m.impl("reset_highway_seeded_", &reset_highway_seeded_);
  m.impl("auto_reset_highway_", &auto_reset_highway_);
  m.impl("ix_reset_", &ix_reset_);
  m.impl("ix_reset_parts_", &ix_reset_parts_);
  m.impl("ix_clear_spawn_", &ix_clear_spawn_);
  m.impl("copy_envs_", &copy_envs_);
  m.impl("ix_step_tail_", &ix_step_tail_);
  m.impl("ix_env_step_", &ix_env_step_);
  m.impl("rewards", &rewards);
  m.impl("rewards_ex", &rewards_ex);
  m.impl("rewards_step_", &rewards_step_);
  m.impl("ego_attention_q", &ego_attention_q);
  m.impl("ego_attention_act", &ego_attention_act);
}

TORCH_LIBRARY_IMPL(ttrl, Meta, m) {
  m.impl("simulate_", &meta_none_sim);
  m.impl("road_act_", &meta_none_act);
  m.impl("road_step_", &meta_none_step);
  m.impl("meta_action_", &meta_none_meta);
  m.impl("env_step_", &meta_env_step);
  m.impl("neighbours", &meta_neighbours);
  m.impl("kinematics_obs", &meta_kin);
  m.impl("kinematics_obs_masked_", &meta_kin_masked);
  m.impl("occupancy_grid", &meta_grid);
  m.impl("observe_ttc", &meta_ttc);
  m.impl("observe_lidar", &meta_lidar);
  m.impl("reset_highway_", &meta_reset);
  m.impl("reset_highway_seeded_", &meta_reset_seeded);
  m.impl("auto_reset_highway_", &meta_auto_reset);
  m.impl("ix_reset_", &meta_reset_seeded);
  m.impl("ix_reset_parts_", &meta_ix_reset_parts);
  m.impl("ix_clear_spawn_", &meta_clear_spawn);
  m.impl("copy_envs_", &meta_copy_envs);
  m.impl("ix_step_tail_", &meta_ix_step_tail);
  m.impl("ix_env_step_", &meta_ix_env_step);
  m.impl("rewards", &meta_rewards);
  m.impl("rewards_ex", &meta_rewards_ex);
  m.impl("rewards_step_", &meta_rewards_step);
  m.impl("ego_attention_q", &meta_ego_attention);
  m.impl("ego_attention_act", &meta_ego_attention_act);
}
