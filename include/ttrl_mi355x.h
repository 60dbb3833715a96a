/*
 * ttrl_mi355x.h — C ABI of the MI355X batched straight-highway simulator.
 *
 * This is the drop-in boundary for the reference's env.step() hot path
 * (SURVEY.md §8(b)).  Every entry point works IN PLACE on caller-owned device
 * buffers (plain pointers + sizes; no torch types), enqueues its kernels on the
 * HIP stream passed as `stream` (hipStream_t, may be NULL = default stream), and
 * returns 0 on success or a negative TTRL_E* code.  No entry point allocates,
 * synchronises or keeps global state, so they are reentrant and graph-capturable.
 *
 * Reference interfaces replaced (file:line in ITCAAdvancedTeam/TopoTrafficRL):
 *   ttrl_road_act            Road.act                      ttrl_env/road/road.py:461-464
 *                            (IDMVehicle.act behavior.py:93-137, ControlledVehicle.act controller.py:89-133)
 *   ttrl_road_step           Road.step(dt)                 ttrl_env/road/road.py:466-478
 *                            (Vehicle.step kinematics.py:130-177, handle_collisions objects.py:91-137)
 *   ttrl_meta_action         DiscreteMetaAction.act        ttrl_env/envs/common/action.py:259-260
 *                            (MDPVehicle.act controller.py:295-315)
 *   ttrl_simulate            AbstractEnv._simulate         ttrl_env/envs/common/abstract.py:252-282
 *   ttrl_neighbours          Road.neighbour_vehicles       ttrl_env/road/road.py:480-513
 *   ttrl_observe_kinematics  KinematicObservation.observe  ttrl_env/envs/common/observation.py:233-275
 *                            (Road.close_objects_to road.py:418-447, Vehicle.to_dict kinematics.py:237-261)
 *   ttrl_observe_grid        OccupancyGridObservation.observe observation.py:353-483
 *   ttrl_env_step_grid       AbstractEnv.step with that observation (abstract.py:224-250), one launch
 *   ttrl_reset_highway       scene init: Vehicle.create_random kinematics.py:50-104,
 *                            IDMVehicle.__init__/randomize_behavior behavior.py:48-69
 *   ttrl_rewards             reward/termination template  ttrl_env/envs/intersection_env.py:78-119
 *   ttrl_rewards_step        + the step's time / info     ttrl_env/envs/common/abstract.py:169-186, :239
 *   ttrl_auto_reset_highway  AbstractEnv.reset of the finished envs inside env.step (abstract.py:188-214)
 *   ttrl_ix_reset            IntersectionEnv._reset        ttrl_env/envs/intersection_env.py:135-318
 *                            (_make_vehicles :251-318, _spawn_vehicle :320-348, AbstractEnv.reset abstract.py:188-214)
 *   ttrl_ix_clear_spawn      IntersectionEnv.step tail     ttrl_env/envs/intersection_env.py:135-139
 *                            (_clear_vehicles :350-362, _spawn_vehicle :320-348)
 *   ttrl_ix_step_tail        the step tail + auto-reset from spare scenes (AbstractEnv.reset abstract.py:188-214)
 *   ttrl_ix_env_step         IntersectionEnv.step (intersection_env.py:135-139 over abstract.py:224-250) with
 *                            the auto-reset from spare scenes, in one launch: frames, observation, rewards,
 *                            _clear_vehicles / _spawn_vehicle, the reset's swap
 */
#ifndef TTRL_MI355X_H
#define TTRL_MI355X_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TTRL_ABI_VERSION 8
#define TTRL_MAX_LANES 32
#define TTRL_MAX_ROADS 32
#define TTRL_MAX_NODES 32
#define TTRL_ROUTE_MAX 4
#define TTRL_RNG_WORDS 5
#define TTRL_IX_MAX_INIT 16

enum { TTRL_F32 = 0, TTRL_F64 = 1 };

enum {
  TTRL_OK = 0,
  TTRL_E_ARG = -1,      /* bad argument (null pointer, size out of range, bad dtype) */
  TTRL_E_LAUNCH = -2,   /* HIP launch / runtime error */
  TTRL_E_UNSUPPORTED = -3
};

/* Vehicle kinds (the reference's class per row of road.vehicles). */
enum { TTRL_ABSENT = 0, TTRL_MDP = 1, TTRL_IDM = 2 };

/* DiscreteMetaAction.ACTIONS_ALL (action.py:204). */
enum { TTRL_LANE_LEFT = 0, TTRL_IDLE = 1, TTRL_LANE_RIGHT = 2, TTRL_FASTER = 3, TTRL_SLOWER = 4 };

/* Lane geometry classes (lane.py): StraightLane :159-213, SineLane :235-290, CircularLane :293-350. */
enum { TTRL_LANE_STRAIGHT = 0, TTRL_LANE_SINE = 1, TTRL_LANE_CIRCULAR = 2 };

/*
 * A RoadNetwork (road.py:21-389) flattened in lanes_list() order: lane l belongs to road
 * road[l] = the (from, to) node pair, roads numbered in graph order, and is lane lane_id[l]
 * of that road.  A single road "0"->"1" (RoadNetwork.straight_road_network road.py:291-321,
 * or parallel Sine / Circular lanes) is n_roads = 1; the intersection of IntersectionEnv
 * (intersection_env.py:141-249) is 20 lanes on 20 roads.  Derived geometry (direction,
 * length, heading) is computed on the host with the float64 formulas of the lane
 * constructors.  Shared by every env of a batch.
 */
typedef struct ttrl_lane_table {
  int32_t n_lanes;
  int32_t n_roads;
  double start_x[TTRL_MAX_LANES], start_y[TTRL_MAX_LANES];
  double dir_x[TTRL_MAX_LANES], dir_y[TTRL_MAX_LANES];   /* direction; lateral = (-dir_y, dir_x) */
  double length[TTRL_MAX_LANES], width[TTRL_MAX_LANES];
  double heading[TTRL_MAX_LANES], speed_limit[TTRL_MAX_LANES];
  int32_t forbidden[TTRL_MAX_LANES];
  int32_t type[TTRL_MAX_LANES];                            /* TTRL_LANE_*                      */
  double amplitude[TTRL_MAX_LANES], pulsation[TTRL_MAX_LANES], phase[TTRL_MAX_LANES];  /* SineLane */
  double center_x[TTRL_MAX_LANES], center_y[TTRL_MAX_LANES], radius[TTRL_MAX_LANES];   /* Circular */
  double start_phase[TTRL_MAX_LANES], direction[TTRL_MAX_LANES];  /* direction: +1 clockwise, -1 */
  /* network topology (all zero for a single road: road 0, lane_id = l) */
  int32_t road[TTRL_MAX_LANES];      /* road of each lane                                   */
  int32_t lane_id[TTRL_MAX_LANES];   /* index of the lane within its road                   */
  int32_t priority[TTRL_MAX_LANES];  /* AbstractLane.priority (RegulatedRoad)               */
  int32_t exit_lane[TTRL_MAX_LANES]; /* 1: an "il*" -> "o*" lane (has_arrived, _clear_vehicles) */
  int32_t road_from[TTRL_MAX_ROADS], road_to[TTRL_MAX_ROADS];    /* node ids                */
  int32_t road_first[TTRL_MAX_ROADS], road_n[TTRL_MAX_ROADS];    /* first lane, lane count  */
  int32_t regulation_frequency;      /* RegulatedRoad.REGULATION_FREQUENCY (2); 0 = Road    */
  int32_t _pad2;
} ttrl_lane_table_t;

/*
 * Behaviour constants, explicit per run instead of the reference's mutable class
 * attributes (IDMVehicle behavior.py:20-46, ControlledVehicle controller.py:24-33,
 * Vehicle kinematics.py:21-29, RoadObject objects.py:62, MDPVehicle controller.py:259).
 */
typedef struct ttrl_params {
  double acc_max;                 /* 6.0   ACC_MAX                       */
  double comfort_acc_max;         /* 3.0   COMFORT_ACC_MAX               */
  double comfort_acc_min;         /* -5.0  COMFORT_ACC_MIN               */
  double distance_wanted;         /* 10.0  DISTANCE_WANTED               */
  double time_wanted;             /* 1.5   TIME_WANTED                   */
  double gap_denom;               /* 2*sqrt(-COMFORT_ACC_MAX*COMFORT_ACC_MIN) */
  double politeness;              /* 0.0   POLITENESS                    */
  double lane_change_min_acc_gain;/* 0.2                                 */
  double lane_change_max_braking; /* 2.0   LANE_CHANGE_MAX_BRAKING_IMPOSED */
  double lane_change_delay;       /* 1.0                                 */
  double tau_pursuit;             /* 0.1   TAU_PURSUIT                   */
  double kp_a;                    /* 1/0.6 KP_A                          */
  double kp_heading;              /* 1/0.2 KP_HEADING                    */
  double kp_lateral;              /* 1/0.6 KP_LATERAL                    */
  double max_steering;            /* pi/3  MAX_STEERING_ANGLE            */
  double length;                  /* 5.0   Vehicle.LENGTH                */
  double width;                   /* 2.0   Vehicle.WIDTH                 */
  double diagonal;                /* sqrt(LENGTH^2 + WIDTH^2)            */
  double max_speed;               /* 40.0                                */
  double min_speed;               /* -40.0                               */
  double lane_vehicle_length;     /* 5.0   AbstractLane.VEHICLE_LENGTH   */
  double target_speeds[8];        /* MDPVehicle target speeds (ego)      */
  int32_t n_target_speeds;        /* 3                                   */
  int32_t _pad;
} ttrl_params_t;

/*
 * Batched vehicle state, struct-of-arrays, row-major [n_envs][n_veh], slots in the order of
 * the reference's road.vehicles list.  Real fields have dtype `dtype` (float or double).
 * The ego (env.vehicle) is the env's first TTRL_MDP slot: slot 0 on the highway, after the
 * initial traffic in the intersection.
 * The route / regulation fields may be NULL for a single-road network without regulation.
 */
typedef struct ttrl_state {
  int32_t n_envs;
  int32_t n_veh;
  int32_t dtype;
  int32_t _pad;
  void *x, *y, *heading, *speed, *target_speed, *timer, *delta;
  void *steer, *acc;              /* Vehicle.action {steering, acceleration}   */
  void *impact_x, *impact_y;      /* Vehicle.impact, valid where has_impact    */
  int32_t *lane, *target_lane;    /* lane ids on road ("0","1",id)             */
  int32_t *speed_index;           /* MDPVehicle.speed_index (ego rows)         */
  uint8_t *kind;                  /* TTRL_ABSENT / TTRL_MDP / TTRL_IDM         */
  uint8_t *crashed, *has_impact, *lane_change; /* crashed, impact!=None, enable_lane_change */
  int8_t *route_road, *route_lane; /* [E][N][TTRL_ROUTE_MAX] ControlledVehicle.route entries:
                                      road id, lane id within the road (-1 = None)           */
  int8_t *route_n;                /* route length, -1 = route None                          */
  uint8_t *yielding;              /* RegulatedRoad: is_yielding                             */
  int32_t *reg_steps;             /* [E] RegulatedRoad.steps (frames since the road was made) */
  uint64_t *rng;                  /* [E][TTRL_RNG_WORDS] AbstractEnv.np_random, numpy Generator(PCG64):
                                     {state_hi, state_lo, inc_hi, inc_lo, has_uint32 << 32 | uinteger};
                                     may be NULL unless a kernel draws from it (intersection
                                     spawns, numpy-order shuffled observation)                  */
} ttrl_state_t;

/* KinematicObservation config (observation.py:159-196).  Feature codes below. */
enum {
  TTRL_F_PRESENCE = 0, TTRL_F_X, TTRL_F_Y, TTRL_F_VX, TTRL_F_VY, TTRL_F_HEADING,
  TTRL_F_COS_H, TTRL_F_SIN_H, TTRL_F_COS_D, TTRL_F_SIN_D, TTRL_F_LONG_OFF,
  TTRL_F_LAT_OFF, TTRL_F_ANG_OFF, TTRL_F_ON_ROAD, TTRL_N_FEATURES
};

typedef struct ttrl_kin_cfg {
  int32_t vehicles_count;         /* V rows                                     */
  int32_t n_features;             /* F columns                                  */
  int32_t features[TTRL_N_FEATURES];
  int32_t absolute, normalize, clip, see_behind;
  int32_t order_shuffled;         /* 0 sorted, 1 shuffled (Philox, seed+offset),
                                     2 shuffled with the env's np_random (state.rng), as the reference */
  int32_t _pad;
  double range_lo[TTRL_N_FEATURES], range_hi[TTRL_N_FEATURES];
  int32_t has_range[TTRL_N_FEATURES];
  double perception_distance;     /* AbstractEnv.PERCEPTION_DISTANCE = 200      */
  uint64_t shuffle_seed, shuffle_offset;
} ttrl_kin_cfg_t;

/* OccupancyGridObservation config (observation.py:285-326). */
typedef struct ttrl_grid_cfg {
  int32_t n_features;
  int32_t features[TTRL_N_FEATURES];
  int32_t shape_x, shape_y;       /* floor((max-min)/step)                      */
  int32_t clip;
  double grid_min_x, grid_min_y, step_x, step_y;
  double range_lo[TTRL_N_FEATURES], range_hi[TTRL_N_FEATURES];
  int32_t has_range[TTRL_N_FEATURES];
  double lane_perception_distance;/* 100 (fill_road_layer_by_lanes)             */
} ttrl_grid_cfg_t;

/* TimeToCollisionObservation config (observation.py:114-151, finite_mdp.py:104-167). */
typedef struct ttrl_ttc_cfg {
  int32_t horizon_bins;           /* int(horizon * policy_frequency) (10)       */
  int32_t obs_lanes, obs_speeds;  /* 3, 3 (observation.py:139, :146); 0, 0: the raw
                                     compute_ttc_grid [speeds][lanes][horizon_bins]
                                     (AbstractEnv.to_finite_mdp, finite_mdp.py:48)  */
  int32_t _pad;
  double time_quantization;       /* 1 / policy_frequency                       */
} ttrl_ttc_cfg_t;

/* LidarObservation config (observation.py:677-768). */
typedef struct ttrl_lidar_cfg {
  int32_t cells;                  /* 16 (<= 64)                                 */
  int32_t normalize;              /* divide by maximum_range                    */
  double maximum_range;           /* 60                                         */
} ttrl_lidar_cfg_t;

/* Highway scene generator config. */
typedef struct ttrl_reset_cfg {
  int32_t n_vehicles;             /* vehicles actually spawned per env (<= n_veh) */
  int32_t ego_lane;               /* 1                                          */
  double ego_x, ego_speed;        /* 50, 25                                     */
  double speed_lo, speed_hi;      /* 0.7*limit, 0.8*limit (host float64)        */
  double spacing;                 /* 1                                          */
  double density_factor;          /* exp(-5/40 * n_lanes) (host float64)        */
  double delta_lo, delta_hi;      /* IDMVehicle.DELTA_RANGE                     */
  int32_t lane_change;            /* enable_lane_change for IDM vehicles        */
  int32_t _pad;
} ttrl_reset_cfg_t;

/* Reward / termination config (IntersectionEnv._agent_reward template). */
typedef struct ttrl_reward_cfg {
  double collision_reward, high_speed_reward, speed_lo, speed_hi;
  int32_t normalize_reward, offroad_terminal;
  double duration;                /* truncation time [s]                        */
  double arrived_reward;          /* reward once has_arrived (intersection_env.py:85) */
  double exit_distance;           /* has_arrived exit_distance (25, :364-369)   */
} ttrl_reward_cfg_t;

/*
 * IntersectionEnv scene (intersection_env.py:17-55 default_config, :251-362).  Corners c = 0..3
 * name the nodes "o"c / "ir"c / "il"c of _make_road; node ids are those of the lane table.
 */
typedef struct ttrl_ix_cfg {
  int32_t initial_vehicle_count;  /* 10                                          */
  int32_t warmup_frames;          /* simulation_steps (3) * simulation_frequency  */
  double warmup_dt;               /* 1 / simulation_frequency                    */
  double init_longitudinal[TTRL_IX_MAX_INIT]; /* np.linspace(0, 80, n)[t]        */
  double spawn_probability;       /* 0.6                                         */
  double spawn_offset;            /* 5: longitudinal + 5 + normal() * deviation  */
  double spawn_speed;             /* 8: 8 + normal() * deviation                 */
  double spawn_clear_distance;    /* 15                                          */
  double challenger_longitudinal; /* 60                                          */
  double challenger_position_deviation, challenger_speed_deviation;  /* 0.1, 0   */
  double delta_lo, delta_hi;      /* IDMVehicle.DELTA_RANGE (randomize_behavior) */
  int32_t n_corners;              /* 4                                           */
  int32_t entry_lane[4];          /* lane ("o"c, "ir"c, 0)                       */
  int32_t exit_node[4];           /* node "o"c                                   */
  int32_t ego_lane;               /* ("o0", "ir0", 0)                            */
  int32_t ego_destination;        /* corner of config["destination"]; -1: integers(1, 4) */
  double ego_longitudinal, ego_deviation;  /* lane.position(60 + 5 * normal(1), 0) */
  double ego_heading_s;           /* heading_at(60)                              */
  double ego_speed;               /* ego lane speed limit                        */
  double ego_clear_distance;      /* 20 ("prevent early collisions")            */
  double leave_margin;            /* 4 * Vehicle.LENGTH (_clear_vehicles)        */
  /* RoadNetwork.shortest_path(node, exit_node[c]) (road.py:159-188) as road ids, -1 padded;
   * path_len 0 = no path (plan_route_to then keeps route = [lane_index]). */
  int8_t path_road[TTRL_MAX_NODES][4][TTRL_ROUTE_MAX - 1];
  int8_t path_len[TTRL_MAX_NODES][4];
} ttrl_ix_cfg_t;

int ttrl_abi_version(void);

/* Ego meta-action (frame 0 of a policy step); actions [n_envs] int32. */
int ttrl_meta_action(const ttrl_state_t* s, const ttrl_lane_table_t* road,
                     const ttrl_params_t* p, const int32_t* actions, void* stream);
/* One Road.act() over every env. */
int ttrl_road_act(const ttrl_state_t* s, const ttrl_lane_table_t* road,
                  const ttrl_params_t* p, void* stream);
/* One Road.step(dt) over every env: kinematics + lane update + collisions. */
int ttrl_road_step(const ttrl_state_t* s, const ttrl_lane_table_t* road,
                   const ttrl_params_t* p, double dt, void* stream);
/* Fused AbstractEnv._simulate: `frames` x (meta-action at frame 0 if actions
 * != NULL, Road.act, Road.step(dt)) with the state resident on chip. */
int ttrl_simulate(const ttrl_state_t* s, const ttrl_lane_table_t* road,
                  const ttrl_params_t* p, const int32_t* actions, int32_t frames,
                  double dt, void* stream);
/* AbstractEnv.step (abstract.py:224-250) in one launch: ttrl_simulate, then from the on-chip final
 * state the Kinematics observation (ttrl_observe_kinematics; skipped when obs_cfg is NULL) and the
 * step tail of ttrl_rewards_step (time += time_inc, reward, terminated, truncated, components, the
 * info's ego speed / crashed; skipped when reward_cfg is NULL).  Same outputs as the separate
 * calls, on every road (the intersection's network with routes included, where an
 * order_shuffled == 2 observation draws from state.rng as ttrl_observe_kinematics does).
 * order (optional, device [n_envs] int32): a permutation of the envs, the order in which the
 * launch's workgroups take them on a road network (as ttrl_ix_step_tail writes it: heaviest
 * first); a dispatch order only -- every output is the same with or without it; other roads
 * ignore it.  It must name every env at most once (a repeated env would be written by two
 * workgroups; not checked, that would need a host sync); a negative entry is an idle slot.
 * action_lut (host, n_action_lut <= 8 meta-action codes; n_action_lut 0: none): actions
 * are action indices, mapped to their codes in the launch (DiscreteMetaAction's index -> action
 * name -> code), so a non-identity action set needs no lookup launch; an index outside the table
 * is no meta-action. */
int ttrl_env_step(const ttrl_state_t* s, const ttrl_lane_table_t* road, const ttrl_params_t* p,
                  const int32_t* actions, int32_t frames, double dt,
                  const ttrl_kin_cfg_t* obs_cfg, float* obs, int32_t* obs_ids,
                  const ttrl_reward_cfg_t* reward_cfg, double* time, double time_inc,
                  float* reward, uint8_t* terminated, uint8_t* truncated, float* components,
                  void* ego_speed, uint8_t* ego_crashed, const int32_t* order, const int32_t* action_lut,
                  int32_t n_action_lut, void* stream);
/* ttrl_env_step with an OccupancyGridObservation (observation.py:353-483) of the final state
 * instead of the Kinematics one: grid [E][F][shape_x][shape_y] float32, as ttrl_observe_grid
 * writes it after ttrl_env_step.  On a straight road of 64 / 128 vehicle slots the step's own
 * launch writes it from its LDS view (one launch); elsewhere the two launches run in turn. */
int ttrl_env_step_grid(const ttrl_state_t* s, const ttrl_lane_table_t* road, const ttrl_params_t* p,
                       const int32_t* actions, int32_t frames, double dt,
                       const ttrl_grid_cfg_t* grid_cfg, float* grid,
                       const ttrl_reward_cfg_t* reward_cfg, double* time, double time_inc,
                       float* reward, uint8_t* terminated, uint8_t* truncated, float* components,
                       void* ego_speed, uint8_t* ego_crashed, const int32_t* action_lut,
                       int32_t n_action_lut, void* stream);
/* Road.neighbour_vehicles(v, lane) for every vehicle; query_lane [E*N] int32
 * (-1 = the vehicle's own lane).  front/rear [E*N] int32 vehicle index or -1. */
int ttrl_neighbours(const ttrl_state_t* s, const ttrl_lane_table_t* road,
                    const int32_t* query_lane, int32_t* front, int32_t* rear, void* stream);
/* Kinematics observation of the ego: out [E][V][F] float32, ids [E][V-1] int32 (-1 pad). */
int ttrl_observe_kinematics(const ttrl_state_t* s, const ttrl_lane_table_t* road,
                            const ttrl_params_t* p, const ttrl_kin_cfg_t* cfg,
                            float* out, int32_t* ids, void* stream);
/* As ttrl_observe_kinematics, for the envs with mask[e] != 0 only (mask NULL: all); the other
 * envs' rows and np_random are left untouched (masked auto-reset re-observation). */
int ttrl_observe_kinematics_masked(const ttrl_state_t* s, const ttrl_lane_table_t* road,
                                   const ttrl_params_t* p, const ttrl_kin_cfg_t* cfg, const uint8_t* mask,
                                   float* out, int32_t* ids, void* stream);
/* Occupancy grid of the ego: out [E][F][shape_x][shape_y] float32. */
int ttrl_observe_grid(const ttrl_state_t* s, const ttrl_lane_table_t* road,
                      const ttrl_params_t* p, const ttrl_grid_cfg_t* cfg,
                      float* out, void* stream);
/* Time-to-collision grid of the ego (compute_ttc_grid finite_mdp.py:104-167 + the lane / speed
 * windows of TimeToCollisionObservation.observe observation.py:126-151):
 * out [E][obs_speeds][obs_lanes][horizon_bins] float32. */
int ttrl_observe_ttc(const ttrl_state_t* s, const ttrl_lane_table_t* road,
                     const ttrl_params_t* p, const ttrl_ttc_cfg_t* cfg, float* out, void* stream);
/* Lidar of the ego (LidarObservation.trace observation.py:704-752): out [E][cells][2] float32
 * {distance, relative speed along the ray}, divided by maximum_range if normalize. */
int ttrl_observe_lidar(const ttrl_state_t* s, const ttrl_lane_table_t* road,
                       const ttrl_params_t* p, const ttrl_lidar_cfg_t* cfg, float* out, void* stream);
/* Scene generation, bit-exact with numpy.random.Generator(PCG64) draws:
 * pcg [E][4] uint64 = {state_hi, state_lo, inc_hi, inc_lo} per env (from
 * SeedSequence on the host); writes all state rows (slots >= n_vehicles absent). */
int ttrl_reset_highway(const ttrl_state_t* s, const ttrl_lane_table_t* road,
                       const ttrl_params_t* p, const ttrl_reset_cfg_t* cfg,
                       const uint64_t* pcg, void* stream);
/* Scene init seeded on the device: env e draws from numpy's
 * default_rng(SeedSequence(entropy[e*n_words .. e*n_words+n_words-1])) (each uint32 word one
 * entropy int), replacing AbstractEnv.reset (abstract.py:188-214) for the envs with
 * mask[e] != 0 (mask NULL: all envs).  No host round trip: the masked auto-reset path. */
int ttrl_reset_highway_seeded(const ttrl_state_t* s, const ttrl_lane_table_t* road,
                              const ttrl_params_t* p, const ttrl_reset_cfg_t* cfg,
                              const uint32_t* entropy, int32_t n_words, const uint8_t* mask,
                              void* stream);
/* VecHighwayEnv.step's auto-reset in one launch: done[e] = terminated[e] | truncated[e]; each done
 * env increments entropy[e][episode_word] (its episode counter), is regenerated as by
 * ttrl_reset_highway_seeded from the incremented words (n_words <= 8) and gets time[e] = 0. */
int ttrl_auto_reset_highway(const ttrl_state_t* s, const ttrl_lane_table_t* road,
                            const ttrl_params_t* p, const ttrl_reset_cfg_t* cfg, uint32_t* entropy,
                            int32_t n_words, int32_t episode_word, const uint8_t* terminated,
                            const uint8_t* truncated, double* time, uint8_t* done, void* stream);
/* Host helper: the initial PCG64 state {state_hi, state_lo, inc_hi, inc_lo} of
 * np.random.PCG64(SeedSequence(entropy words)) (numpy bit_generator.pyx / pcg64.h). */
int ttrl_seed_pcg64(const uint32_t* entropy, int32_t n_words, uint64_t* state4);
/* EgoAttention Q-values for config 5 (ttrl_agent models.py:157-312, ego_attention_2h.json), float32:
 * obs [batch][n_entities][n_features] (feature 0 = presence), q [batch][n_actions].
 * weights: one packed buffer, every matrix transposed from torch's Linear.weight to [in][out]
 * (row-major), in this order:
 *   ego_embedding  W1 [F][64], b1 [64], W2 [64][64], b2 [64]
 *   others_embedding W1 [F][64], b1 [64], W2 [64][64], b2 [64]
 *   attention value_all [64][64], key_all [64][64], query_ego [64][64], attention_combine [64][64]
 *   output_layer   W1 [64][64], b1 [64], W2 [64][64], b2 [64], predict W [64][A], b [A]
 * ttrl_ego_attention_sizes returns the packed length (floats) and sets *scratch_floats to the
 * scratch the forward needs (caller-allocated device memory). */
int64_t ttrl_ego_attention_sizes(int32_t n_features, int32_t n_actions, int32_t batch, int32_t n_entities,
                                 int64_t* scratch_floats);
int ttrl_ego_attention_q(const float* obs, int32_t batch, int32_t n_entities, int32_t n_features,
                         int32_t heads, const float* weights, int32_t n_actions, float* scratch, float* q,
                         void* stream);
/* AbstractDQNAgent.act (dqn/abstract.py:65-83) with EpsilonGreedy (epsilon_greedy.py:32-48) for a
 * batch, in the same launch as the forward above: q [batch][n_actions] (as ttrl_ego_attention_q)
 * and actions [batch] int64 = np.argmax(q[e]) (first maximum), replaced with probability epsilon by
 * a uniform action -- the reference's action distribution.  The draws are Philox4x32-10 keyed on
 * seed, counter (env_offset + e, step), env_offset the global id of row 0 (a rank's shard offset):
 * reproducible per (seed, global env, step) whatever the batch split, and distinct across the
 * data-parallel shards of one seed.  epsilon_dev /
 * step_dev (device scalars, optional) override epsilon / step, for captured graphs.  epsilon must
 * lie in [0, 1].  actions / actions32: the same actions as int64 and as int32 (the env's action
 * index type, ttrl_simulate's `actions`); either may be NULL, not both. */
int ttrl_ego_attention_act(const float* obs, int32_t batch, int32_t n_entities, int32_t n_features,
                           int32_t heads, const float* weights, int32_t n_actions, float epsilon,
                           const float* epsilon_dev, uint64_t seed, int64_t step, const int64_t* step_dev,
                           int64_t env_offset, float* q, int64_t* actions, int32_t* actions32, void* stream);
/* IntersectionEnv._reset for the envs with mask[e] != 0 (mask NULL: all): np_random =
 * default_rng(SeedSequence(entropy[e][0..n_words-1])) into state.rng, then _make_vehicles:
 * initial spawns, warmup_frames of Road.act/step (RegulatedRoad), the challenger, the ego
 * MDPVehicle (appended after the traffic) and the removal of vehicles near it.  Requires the
 * network fields and state.rng.  Vehicles beyond n_veh slots are dropped (draws still made). */
int ttrl_ix_reset(const ttrl_state_t* s, const ttrl_lane_table_t* road, const ttrl_params_t* p,
                  const ttrl_ix_cfg_t* cfg, const uint32_t* entropy, int32_t n_words, const uint8_t* mask,
                  void* stream);
/* ttrl_ix_reset in parts, each over its own env mask (NULL: all): TTRL_IX_BEGIN (seeding and the
 * initial spawns, from entropy), TTRL_IX_WARMUP (warm_frames of the warm-up frames -- consecutive
 * calls continue the same warm-up), TTRL_IX_FINISH (the challenger, the ego and the removals).
 * ttrl_ix_reset == all three over one mask with warm_frames = cfg->warmup_frames.  Lets a caller
 * spread a reset's warm-up over several steps, the chunks of different resets in one launch. */
enum { TTRL_IX_BEGIN = 1, TTRL_IX_WARMUP = 2, TTRL_IX_FINISH = 4 };
int ttrl_ix_reset_parts(const ttrl_state_t* s, const ttrl_lane_table_t* road, const ttrl_params_t* p,
                        const ttrl_ix_cfg_t* cfg, int32_t parts, const uint32_t* entropy, int32_t n_words,
                        const uint8_t* begin_mask, const uint8_t* warm_mask, int32_t warm_frames,
                        const uint8_t* finish_mask, void* stream);
/* Copy every row of the envs with mask[e] != 0 (all fields, per-env route / regulation / rng
 * words included) from src to dst, which have the same shape and dtype: swapping in scenes reset
 * ahead of time (the intersection's double-buffered auto-reset). */
int ttrl_copy_envs(const ttrl_state_t* dst, const ttrl_state_t* src, const uint8_t* mask, void* stream);
/* IntersectionEnv.step tail after the observation and reward: _clear_vehicles (list order kept),
 * then _spawn_vehicle(spawn_probability) drawing from state.rng; envs with mask[e] != 0. */
int ttrl_ix_clear_spawn(const ttrl_state_t* s, const ttrl_lane_table_t* road, const ttrl_params_t* p,
                        const ttrl_ix_cfg_t* cfg, const uint8_t* mask, void* stream);
/* VecIntersectionEnv.step after ttrl_env_step (fused frames, observation, rewards), with the
 * auto-reset from scenes reset ahead of time, in one launch.  spare: K * E rows, K in [2, 16] (slot
 * q of env e is row q * E + e), reset by ttrl_ix_reset from spare_entropy.  An env with
 * terminated | truncated == 0 runs the IntersectionEnv.step tail (as ttrl_ix_clear_spawn) and
 * copies its observation row obs_in -> obs_out; a finished env instead takes the spare row of slot
 * spare_parity[e] (every field, rng and regulation words included), moves spare_parity[e] to the
 * next slot (mod K), adds 1 to its episode word entropy[e][n_words - 1] and K to
 * spare_entropy[row][n_words - 1], zeroes time[e] and writes its first observation into obs_out /
 * obs_ids_out (obs_cfg: Kinematics, n_veh <= 64).  done[E] = terminated | truncated;
 * spare_mask[K * E] flags the consumed spare rows (to be reset again).
 * live_count (optional, one int64 on the device): += the vehicles present in the E envs after
 * the tail -- the next step's live vehicles, counted without a launch of its own (the
 * intersection bench's live vehicle-steps).  order (optional, device [2 * n_envs] int32, the
 * first n_envs initialised to any permutation of the envs): receives in [0, n_envs) the next
 * ttrl_env_step's dispatch order -- the envs grouped as that launch's workgroups hold them,
 * groups sorted by their live vehicles, heaviest first; [n_envs, 2 n_envs) is its scratch.
 * Reference: intersection_env.py:135-139, :350-362, :320-348; abstract.py:188-214. */
int ttrl_ix_step_tail(const ttrl_state_t* s, const ttrl_lane_table_t* road, const ttrl_params_t* p,
                      const ttrl_ix_cfg_t* cfg, const ttrl_state_t* spare, const uint8_t* terminated,
                      const uint8_t* truncated, uint8_t* spare_parity, uint32_t* entropy, uint32_t* spare_entropy,
                      int32_t n_words, double* time, uint8_t* done, uint8_t* spare_mask,
                      const ttrl_kin_cfg_t* obs_cfg, const float* obs_in, float* obs_out, const int32_t* obs_ids_in,
                      int32_t* obs_ids_out, int64_t* live_count, int32_t* order, void* stream);
/* VecIntersectionEnv.step with the auto-reset from spare scenes in one launch (ABI 7): ttrl_env_step
 * followed by ttrl_ix_step_tail, fused, on a road network of <= 64 slots (one wavefront per
 * workgroup).  From the on-chip final state: the Kinematics observation (obs_cfg -> obs / obs_ids)
 * and the step tail (time += time_inc, reward, terminated, truncated, components, ego speed /
 * crashed) as ttrl_env_step; then an env that goes on (terminated | truncated == 0) runs
 * IntersectionEnv.step's tail as ttrl_ix_clear_spawn does (_clear_vehicles, then _spawn_vehicle
 * drawing from state.rng after the observation's shuffle) and keeps its observation row as its
 * next one (obs_next / ids_next), while a finished env takes its spare scene and counters and has
 * its new first observation written to obs_next / ids_next -- spare, spare_parity, entropy,
 * spare_entropy, n_words, done, spare_mask, live_count and order exactly as ttrl_ix_step_tail takes
 * them (the next dispatch order is written after the launch).  The spare rows an env may take must
 * be ready when the launch starts (VecIntersectionEnv keeps one more spare slot for that).  Bit for
 * bit ttrl_env_step + ttrl_ix_step_tail.  Reference: intersection_env.py:135-139, :320-362;
 * abstract.py:188-250. */
int ttrl_ix_env_step(const ttrl_state_t* s, const ttrl_lane_table_t* road, const ttrl_params_t* p,
                     const ttrl_ix_cfg_t* cfg, const int32_t* actions, int32_t frames, double dt,
                     const ttrl_kin_cfg_t* obs_cfg, float* obs, int32_t* obs_ids, float* obs_next, int32_t* ids_next,
                     const ttrl_reward_cfg_t* reward_cfg, double* time, double time_inc, float* reward,
                     uint8_t* terminated, uint8_t* truncated, float* components, void* ego_speed,
                     uint8_t* ego_crashed, const ttrl_state_t* spare, uint8_t* spare_parity, uint32_t* entropy,
                     uint32_t* spare_entropy, int32_t n_words, uint8_t* done, uint8_t* spare_mask, int32_t* order,
                     const int32_t* action_lut, int32_t n_action_lut, int64_t* live_count, void* stream);
/* Per-env reward [E] float32, terminated/truncated [E] uint8, given time [E] float64, for the
 * env's controlled vehicle (its first TTRL_MDP slot). */
int ttrl_rewards(const ttrl_state_t* s, const ttrl_lane_table_t* road,
                 const ttrl_reward_cfg_t* cfg, const double* time, float* reward,
                 uint8_t* terminated, uint8_t* truncated, void* stream);
/* As ttrl_rewards, plus the per-objective terms of IntersectionEnv._agent_rewards
 * (intersection_env.py:95-104) in components [E][4] float32: collision_reward (crashed),
 * high_speed_reward (clipped lmap of the speed), arrived_reward, on_road_reward. */
int ttrl_rewards_ex(const ttrl_state_t* s, const ttrl_lane_table_t* road,
                    const ttrl_reward_cfg_t* cfg, const double* time, float* reward,
                    uint8_t* terminated, uint8_t* truncated, float* components, void* stream);
/* The env.step tail in one launch: time[E] += time_inc (AbstractEnv.step abstract.py:239; 0 leaves
 * time untouched), then ttrl_rewards_ex, and -- when ego_speed / ego_crashed are given (both or
 * neither) -- the info's speed [E] (the state's dtype) and crashed [E] uint8 of the controlled
 * vehicle (abstract.py:169-186; slot 0 for an env without one). */
int ttrl_rewards_step(const ttrl_state_t* s, const ttrl_lane_table_t* road,
                      const ttrl_reward_cfg_t* cfg, double* time, double time_inc, float* reward,
                      uint8_t* terminated, uint8_t* truncated, float* components, void* ego_speed,
                      uint8_t* ego_crashed, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* TTRL_MI355X_H */
