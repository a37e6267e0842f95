/*
 * plantos_batch.h -- C-ABI of the MI355X-native batched PlantOSEnv step/reset.
 *
 * Drop-in boundary.  The reference has no native FFI: its
 * boundary is two Python protocols, and every entry point below replaces one of
 * them for a whole batch of N envs resident in HBM:
 *
 *   pe_create       PlantOSEnv.__init__              plantos_env.py:25-123
 *                   + DummyVecEnv(env_fns)           A2C_training.py:216-218
 *   pe_reset        PlantOSEnv.reset                 plantos_env.py:125-158
 *                   (map generation _generate_map    plantos_env.py:338-372)
 *   pe_step         PlantOSEnv.step                  plantos_env.py:160-183
 *                   + DummyVecEnv.step_wait auto-reset (SB3)
 *   pe_get_info     PlantOSEnv._get_info             plantos_env.py:317-336
 *   pe_get_state /  the state tuple MCTS clones      mcts_custom_trainer.py:236-241
 *   pe_set_state    (+ CurriculumWrapper visit_counts injection, A2C_training.py:88-93)
 *   pe_load_maps    reset() with a host-supplied layout (seed-exact CPython stream mode)
 *   pe_seed         VecEnv.seed / reset(seed=...)    (the reference ignores it for maps)
 *   pe_destroy      PlantOSEnv.close                 plantos_env.py:522-528
 *   pe_mcts_*       MCTS.search for every env at once mcts_custom_trainer.py:72-243
 *
 * Conventions
 *  - Every array argument is a DEVICE pointer (caller-owned, e.g. a torch tensor on
 *    the handle's device), row-major, env index outermost.  Only the handle's state
 *    is owned by the library.
 *  - Calls are asynchronous on `stream` (a hipStream_t passed as void*; NULL = the
 *    default stream).  They return PE_OK or a negative PE_ERR_* code; the message of
 *    the last failure on the calling thread is pe_last_error().
 *  - A handle is bound to one device and is not re-entrant.
 *  - No CPU fallback: if the HIP runtime or a gfx950 device is unavailable, pe_create
 *    fails with PE_ERR_DEVICE.
 */
#ifndef PLANTOS_BATCH_H
#define PLANTOS_BATCH_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PE_ABI_VERSION 4

enum pe_status {
    PE_OK = 0,
    PE_ERR_ARG = -1,      /* bad argument / config (Python: ValueError)            */
    PE_ERR_DEVICE = -2,   /* HIP runtime / device failure                          */
    PE_ERR_NOMEM = -3,    /* device allocation failed                              */
    PE_ERR_NOROOM = -4,   /* map generation had no room (plantos_env.py:360-364)  */
};

/* Per-env scalar slots of the canonical state (pe_get_state / pe_set_state), int32. */
enum pe_scalar {
    PE_S_X = 0,        /* rover_pos[0] (row)          plantos_env.py:96  */
    PE_S_Y = 1,        /* rover_pos[1] (column)                           */
    PE_S_STEP = 2,     /* step_count                  plantos_env.py:119 */
    PE_S_COLL = 3,     /* total_collisions            plantos_env.py:123 */
    PE_S_COLLIDED = 4, /* collided_with_wall          plantos_env.py:121 */
    PE_S_BONUS = 5,    /* completion_bonus_given      plantos_env.py:122 */
    PE_S_POISONED = 6, /* bit0: root env would raise TypeError (watering a hydrated
                          plant, plantos_env.py:217-220); bit1: action < -4 (IndexError);
                          bit2: last reset had no room (ValueError)                */
    PE_S_EPISODE = 7,  /* number of resets so far (device-rng stream index)        */
    PE_NSCAL = 8
};

/* pe_get_info columns, int32 (plantos_env.py:317-336). */
enum pe_info {
    PE_I_X = 0, PE_I_Y, PE_I_THIRSTY, PE_I_HYDRATED, PE_I_TOTAL_PLANTS, PE_I_STEP,
    PE_I_EXPLORED, PE_I_TOTAL_CELLS, PE_I_COLLIDED, PE_I_COLLISIONS, PE_I_POISONED,
    PE_NINFO
};

/* Cell codes of the canonical grid (obstacles set + plants dict, plantos_env.py:97-98). */
enum pe_cell { PE_EMPTY = 0, PE_OBSTACLE = 1, PE_HYDRATED = 2, PE_THIRSTY = 3 };

typedef struct pe_config {
    int32_t abi_version;        /* = PE_ABI_VERSION */
    int32_t grid_size;          /* G, plantos_env.py:25 (device: 1..128)        */
    int32_t num_plants;         /* P                                            */
    int32_t num_obstacles;      /* O -> O/3 clusters, plantos_env.py:341        */
    int32_t lidar_range;        /* R (device: 1..64)                            */
    int32_t lidar_channels;     /* C (device: the lane-per-env kernels' [64 x D] f32 LDS
                                   obs tile + 2CR bytes of ray offsets within 160 KiB:
                                   C <= 120 at R <= 7, fewer rays above)         */
    int32_t max_steps;          /* 1000, plantos_env.py:120                     */
    int32_t autoreset;          /* 1: pe_step resets done envs (DummyVecEnv)    */
    double thirsty_plant_prob;  /* 0.7, plantos_env.py:26                       */
    double r_goal, r_mistake, r_invalid, r_water_empty; /* plantos_env.py:76-79 */
    double r_step, r_exploration, r_revisit, r_complete; /* plantos_env.py:80-83 */
    uint64_t seed;              /* device-rng key (Philox4x32-10)               */
    uint32_t env_id_offset;     /* global id of env 0 (sharding across GPUs)    */
    int32_t map_generation_algo; /* PE_MAP_ORIGINAL (0, plantos_env.py:338-372) or
                                    PE_MAP_MAZE (the fork's map_generation_algo='maze',
                                    gradio-app/plantos_env_new.py:355-358, 408-604; G >= 7) */
    /* Auto-reset tuning (speed only: every setting gives the same results).  -1 = the
     * library's choice for the geometry (pe_default_config sets -1).              */
    int32_t coop_max_done;      /* a step-kernel block resets up to this many done envs
                                   wave-cooperatively, more one lane per env; 0 = always
                                   one lane per env                                 */
    int32_t prefetch_every;     /* steps between the launches that generate next-episode
                                   maps ahead of time; 0 = no prefetched resets       */
    int32_t obs_codes;          /* 1: the step kernel keeps the obs as byte codes (one byte
                                   per value, every value is one of < 256 table floats):
                                   pe_step_codes writes them (5C+27 B per env instead of
                                   4(5C+27)), pe_expand_obs_codes turns them into floats.
                                   Geometries whose step kernel is a sector kernel that
                                   can hold a byte-coded tile: C = 16 / R = 6 with G <= 20,
                                   C = 64 / R = 6, and every geometry of the runtime-(C, R)
                                   sector kernel (4 <= C <= 64, 2 <= R <= 14, no compile-
                                   time kernel), and the far sector kernel's C = 64 / R = 32
                                   with 96 < G + 2R <= 128; pe_create fails with PE_ERR_ARG
                                   elsewhere.
                                   pe_step still writes f32 obs on such a handle.
                                   0 (default): off                                     */
    int32_t reserved[3];
} pe_config;

enum pe_map_algo { PE_MAP_ORIGINAL = 0, PE_MAP_MAZE = 1 };

typedef struct pe_handle pe_handle;

/* Fill `c` with the reference defaults for the given geometry
 * (plantos_env.py:25-27, 76-83, 120). */
void pe_default_config(pe_config* c, int32_t grid_size, int32_t num_plants, int32_t num_obstacles,
                       int32_t lidar_range, int32_t lidar_channels);

/* Observation length 5*C + 2 + 25 (plantos_env.py:55-57). */
int32_t pe_obs_dim(const pe_config* c);

/* Allocate the SoA state for n_envs envs on `device`. All envs start reset (episode 0). */
int pe_create(const pe_config* c, int32_t device, int32_t n_envs, pe_handle** out);
int pe_destroy(pe_handle* h);

/* Re-key the device RNG (and optionally zero the episode counters), ordered on
 * `stream` after the work already queued there (step / prefetch kernels). */
int pe_seed(pe_handle* h, uint64_t seed, int32_t reset_episode_counters, void* stream);

/* Reset the envs whose mask byte is non-zero (all envs when mask == NULL) with the
 * device-rng map generator, then write obs[n_envs, D] for ALL envs (reset ones get
 * their fresh obs, the others their current obs). */
int pe_reset(pe_handle* h, const uint8_t* mask_or_null, float* obs, void* stream);

/* One step of every env.
 *   actions      int32[n] or int64[n] (action_bytes = 4 or 8); 0..3 move N/E/S/W, >=4 water
 *   obs          f32[n, D]   post-step obs (post-reset obs for done envs when autoreset)
 *   reward       f32[n]      reward (computed in f64 like the reference, cast once)
 *   terminated   u8[n], truncated u8[n]
 *   terminal_obs f32[n, D] or NULL: rows of done envs receive the pre-reset obs
 *   episode_return f64[n] or NULL: rows of done envs receive the episode's f64 return
 *   episode_length i32[n] or NULL: rows of done envs receive the episode length
 *   terminal_info  i32[n, PE_NINFO] or NULL: rows of done envs receive _get_info of the
 *                  final (pre-reset) state (DummyVecEnv keeps that step's info dict)
 * Only rows of done envs are written in the four terminal outputs (autoreset on).   */
int pe_step(pe_handle* h, const void* actions, int32_t action_bytes, float* obs, float* reward,
            uint8_t* terminated, uint8_t* truncated, float* terminal_obs_or_null,
            double* episode_return_or_null, int32_t* episode_length_or_null,
            int32_t* terminal_info_or_null, void* stream);

/* pe_step with the obs as byte codes (handles created with obs_codes = 1):
 * obs_codes u8[n, D] instead of f32[n, D]; every other argument as pe_step.  This is
 * the host-boundary form of a sharded job (plantos_amd/shard.py): ranks gather 5C+27 B
 * per env instead of 4(5C+27), and the root expands the codes once. */
int pe_step_codes(pe_handle* h, const void* actions, int32_t action_bytes, uint8_t* obs_codes, float* reward,
                  uint8_t* terminated, uint8_t* truncated, float* terminal_obs_or_null,
                  double* episode_return_or_null, int32_t* episode_length_or_null,
                  int32_t* terminal_info_or_null, void* stream);

/* The float of every obs byte code (table f32[256], host memory; unused codes 0.0). */
int pe_obs_code_table(const pe_handle* h, float* table);

/* Expand `blocks` packed code buffers into contiguous outputs.  Block b starts at
 * src + b * src_stride (bytes, a multiple of 16) and holds codes u8[rows, D], then at
 * the next multiple of 16 bytes reward f32[rows], terminated u8[rows], truncated
 * u8[rows] (the io layout of plantos_amd's code-mode batches); outputs: obs
 * f32[blocks * rows, D] and (each may be NULL) reward f32 / terminated u8 / truncated
 * u8 [blocks * rows], in block order.  Any handle of the same geometry gives the same
 * table (e.g. the root rank's shard expanding every rank's gathered codes). */
int pe_expand_obs_codes(const pe_handle* h, int32_t blocks, int32_t rows, const uint8_t* src, int64_t src_stride,
                        float* obs, float* reward, uint8_t* terminated, uint8_t* truncated, void* stream);

/* info columns (pe_info) for all envs: int32[n, PE_NINFO]. */
int pe_get_info(pe_handle* h, int32_t* info, void* stream);

/* Canonical state, reference terms: cells u8[n,G,G] (pe_cell), visits i32[n,G,G],
 * explored i8[n,G,G] (0/1/2), scalars i32[n,PE_NSCAL].  Any pointer may be NULL
 * (get: skipped; set: that part is left unchanged).  set recomputes derived
 * counters (explored/total cells) from the arrays. Visits are exact int32 counts. */
int pe_get_state(pe_handle* h, uint8_t* cells, int32_t* visits, int8_t* explored, int32_t* scalars,
                 void* stream);
int pe_set_state(pe_handle* h, const uint8_t* cells, const int32_t* visits, const int8_t* explored,
                 const int32_t* scalars, void* stream);

/* Reset k envs (env_index i32[k]) to host-supplied layouts: cells u8[k,G,G] (obstacles
 * and plants only), rover i32[k,2]; then write obs[k, D] for those envs (row j = env
 * env_index[j]).  Used by the seed-exact CPython-stream reset mode. */
int pe_load_maps(pe_handle* h, int32_t k, const int32_t* env_index, const uint8_t* cells,
                 const int32_t* rover, float* obs_k, void* stream);

/* Synthetic benchmark actions: actions[e] = philox(seed, env_id_offset+e, t) % 5. */
int pe_synth_actions(pe_handle* h, uint64_t seed, uint32_t t, int32_t* actions, void* stream);

/* Accumulated error bits OR-ed over all envs since the last call (PE_S_POISONED bit
 * layout); synchronizes the stream. */
int pe_poll_errors(pe_handle* h, int32_t* bits, void* stream);

/* Batched CurriculumWrapper, applied inside pe_step and every reset path.  The
 * reference has two variants of the class, selected by terminate_on_threshold:
 *   1  A2C_training.py:37-109 (defaults 40 / 100 / +10, 3 episodes per maze):
 *      terminated is also reported when exploration_percentage >= the env's
 *      threshold (:101-103);
 *   0  trainingCode.py:24-98 (defaults 30 / 100 / +5, 50 episodes per maze, the
 *      wrapper of its DQN / RecurrentPPO trainers): reaching the threshold only
 *      marks the maze completed (:87-89); the episode runs on until the env itself
 *      terminates or truncates.
 * Both: exploration_percentage >= threshold marks the maze completed; at reset the threshold rises by the
 * increment after a completed maze (capped), a new map starts after a completed
 * maze or max_episodes_per_maze episodes, and otherwise the new episode keeps the
 * previous episode's visit counts (explored map restarted; the reset obs shows the
 * fresh visits, as the wrapper installs them after env.reset()).  The reference's
 * "same maze" intent is not realized there either (reset seeds are ignored).
 * Enabling (re)initializes every env's record (threshold = initial, counters 0),
 * ordered on `stream`. */
int pe_curriculum_enable(pe_handle* h, double initial_threshold, double max_threshold,
                         double threshold_increment, int32_t max_episodes_per_maze,
                         int32_t terminate_on_threshold, void* stream);
int pe_curriculum_disable(pe_handle* h);
/* threshold f64[n]; counters i32[n,4] = episode_count, successful_explorations,
 * episodes_on_current_maze, flags (bit0 maze_completed, bit1 visits carried). Device. */
int pe_curriculum_get(pe_handle* h, double* threshold, int32_t* counters, void* stream);

/* Seed-exact reset layouts (host side): the reference's _generate_map
 * (plantos_env.py:338-372) on CPython's global `random` stream after
 * random.seed(seed), including CPython 3.10 set iteration order, so the maps are
 * the ones the reference produces.  Maps come out in stream order; a DummyVecEnv
 * consumes them in env-index order at reset() and then per step (done envs in
 * index order).  Feed them to pe_load_maps.  pe_pystream_next fails with
 * PE_ERR_NOROOM where the reference raises ValueError (360-364). */
typedef struct pe_pystream pe_pystream;
int pe_pystream_create(const pe_config* c, int64_t seed, pe_pystream** out);
/* next k maps: cells u8[k,G,G] (pe_cell codes), rover i32[k,2]; HOST pointers */
int pe_pystream_next(pe_pystream* s, int32_t k, uint8_t* cells, int32_t* rover);
/* random.getrandbits(32) on the stream (tests pin the number of draws consumed) */
uint32_t pe_pystream_getrandbits32(pe_pystream* s);
int pe_pystream_destroy(pe_pystream* s);

/* Batched MCTS (mcts_custom_trainer.py:72-243): one MCTS.search per env of `h`,
 * every env with its own tree, its own clone of the env state (_copy_env_state
 * :221-243: position, plants, obstacles, explored map, visit counts and step count
 * copied; collision/bonus flags start cleared) and its own np.random stream
 * (numpy legacy RandomState: np.random.seed(int) = MT19937 init_genrand; random()
 * and randint(n) as numpy draws them).  UCB1 selection (:37-60), expansion of a
 * random untried action (:117-125), the 70/30 least-visited-neighbour rollout
 * policy (:141-219, +500 when a rollout ends fully explored), backpropagation and
 * best_action (:62-69) are the reference's, bit for bit.  Sim envs water with the
 * fork's semantics (hydrated plant: R_MISTAKE).  Searches read the live state of
 * `h` and never modify it; they step nothing: apply the actions with pe_step.
 * Scratch: (G*G + 2*max_depth + 2) * 4 + (n_simulations + 1) * 32 + 2504 bytes/env. */
typedef struct pe_mcts pe_mcts;
int pe_mcts_create(pe_handle* h, int32_t n_simulations, double c_param, int32_t max_depth, pe_mcts** out);
int pe_mcts_destroy(pe_mcts* m);
/* np.random.seed(seeds[e]) for env e (HOST array of n, or NULL: base_seed + e). */
int pe_mcts_seed(pe_mcts* m, const uint32_t* seeds, uint32_t base_seed, void* stream);
/* Stream state in numpy's own terms (get_state()[1:3]): key u32[n,624], pos i32[n].
 * HOST arrays; synchronous. */
int pe_mcts_set_rng(pe_mcts* m, const uint32_t* key, const int32_t* pos);
int pe_mcts_get_rng(pe_mcts* m, uint32_t* key, int32_t* pos);
/* One search per env (mask u8[n] or NULL = all): actions i32[n] (masked-out envs
 * untouched); optional root children in insertion order: order i32[n,5] (action,
 * -1 pad), visits i32[n,5], value f64[n,5].  Device pointers. */
int pe_mcts_search(pe_mcts* m, const uint8_t* mask, int32_t* actions, int32_t* root_order, int32_t* root_visits,
                   double* root_value, void* stream);

/* Introspection for tests / benchmarks. */
int32_t pe_num_envs(const pe_handle* h);
int32_t pe_kernel_variant(const pe_handle* h);  /* 0 generic, >0 specialized geometry */
const char* pe_kernel_name(const pe_handle* h);
int32_t pe_prefetch_every(const pe_handle* h);  /* steps between prefetch launches, 0 = off */
uint64_t pe_state_bytes(const pe_handle* h);

const char* pe_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
