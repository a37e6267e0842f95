"""ctypes binding of the C-ABI in include/plantos_batch.h (libplantos_hip.so).

This is the binding a Python maintainer of the reference would add
(INTEGRATION.md): plain pointers and sizes, device buffers owned by torch.
There is no CPU fallback: if the library or a gfx950 device is missing,
loading / pe_create raises.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libplantos_hip.so")
# diagnostics only (tools/ablate.py): load a differently built library
if os.environ.get("PLANTOS_HIP_LIB"):
    LIB_PATH = os.environ["PLANTOS_HIP_LIB"]

PE_ABI_VERSION = 4
PE_OK, PE_ERR_ARG, PE_ERR_DEVICE, PE_ERR_NOMEM, PE_ERR_NOROOM = 0, -1, -2, -3, -4
PE_NSCAL = 8
PE_NINFO = 11
(PE_S_X, PE_S_Y, PE_S_STEP, PE_S_COLL, PE_S_COLLIDED, PE_S_BONUS, PE_S_POISONED, PE_S_EPISODE) = range(8)
(PE_I_X, PE_I_Y, PE_I_THIRSTY, PE_I_HYDRATED, PE_I_TOTAL_PLANTS, PE_I_STEP, PE_I_EXPLORED,
 PE_I_TOTAL_CELLS, PE_I_COLLIDED, PE_I_COLLISIONS, PE_I_POISONED) = range(11)

PE_CELL_EMPTY, PE_CELL_OBSTACLE, PE_CELL_HYDRATED, PE_CELL_THIRSTY = range(4)
PE_MAP_ORIGINAL, PE_MAP_MAZE = 0, 1
MAP_ALGOS = {"original": PE_MAP_ORIGINAL, "maze": PE_MAP_MAZE}


def map_algo_id(name):
    """map_generation_algo of the fork's constructor (plantos_env_new.py:28, 355-358):
    'maze' selects the maze; anything else is 'original', as there."""
    return PE_MAP_MAZE if name == "maze" else PE_MAP_ORIGINAL

# exported symbols (tests/test_capi_symbols.py checks they match include/plantos_batch.h)
EXPORTS = [
    "pe_default_config", "pe_obs_dim", "pe_create", "pe_destroy", "pe_seed", "pe_reset", "pe_step",
    "pe_get_info", "pe_get_state", "pe_set_state", "pe_load_maps", "pe_synth_actions", "pe_poll_errors",
    "pe_num_envs", "pe_kernel_variant", "pe_kernel_name", "pe_prefetch_every", "pe_state_bytes", "pe_last_error",
    "pe_pystream_create", "pe_pystream_next", "pe_pystream_getrandbits32", "pe_pystream_destroy",
    "pe_curriculum_enable", "pe_curriculum_disable", "pe_curriculum_get",
    "pe_mcts_create", "pe_mcts_destroy", "pe_mcts_seed", "pe_mcts_set_rng", "pe_mcts_get_rng", "pe_mcts_search",
    "pe_step_codes", "pe_obs_code_table", "pe_expand_obs_codes",
]


class PEConfig(ctypes.Structure):
    _fields_ = [
        ("abi_version", ctypes.c_int32), ("grid_size", ctypes.c_int32), ("num_plants", ctypes.c_int32),
        ("num_obstacles", ctypes.c_int32), ("lidar_range", ctypes.c_int32), ("lidar_channels", ctypes.c_int32),
        ("max_steps", ctypes.c_int32), ("autoreset", ctypes.c_int32), ("thirsty_plant_prob", ctypes.c_double),
        ("r_goal", ctypes.c_double), ("r_mistake", ctypes.c_double), ("r_invalid", ctypes.c_double),
        ("r_water_empty", ctypes.c_double), ("r_step", ctypes.c_double), ("r_exploration", ctypes.c_double),
        ("r_revisit", ctypes.c_double), ("r_complete", ctypes.c_double), ("seed", ctypes.c_uint64),
        ("env_id_offset", ctypes.c_uint32), ("map_generation_algo", ctypes.c_int32),
        ("coop_max_done", ctypes.c_int32), ("prefetch_every", ctypes.c_int32), ("obs_codes", ctypes.c_int32),
        ("reserved", ctypes.c_int32 * 3),
    ]


class PlantOSNativeError(RuntimeError):
    pass


_lib = None


def lib():
    """Load libplantos_hip.so (built by rl-env_amd/build.py); raise if absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise PlantOSNativeError(
            f"{LIB_PATH} not found: build it with `python rl-env_amd/build.py` "
            "(there is no CPU fallback for the PlantOS hot path)")
    L = ctypes.CDLL(LIB_PATH)
    P, I32, U64, U32 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_uint64, ctypes.c_uint32
    CP = ctypes.POINTER(PEConfig)
    L.pe_default_config.argtypes = [CP, I32, I32, I32, I32, I32]
    L.pe_default_config.restype = None
    L.pe_obs_dim.argtypes = [CP]
    L.pe_obs_dim.restype = I32
    L.pe_create.argtypes = [CP, I32, I32, ctypes.POINTER(P)]
    L.pe_destroy.argtypes = [P]
    L.pe_seed.argtypes = [P, U64, I32, P]
    L.pe_reset.argtypes = [P, P, P, P]
    L.pe_step.argtypes = [P, P, I32, P, P, P, P, P, P, P, P, P]
    if hasattr(L, "pe_step_codes"):  # (ABI 4; an older library loaded for a same-box A/B lacks them)
        L.pe_step_codes.argtypes = [P, P, I32, P, P, P, P, P, P, P, P, P]
        L.pe_obs_code_table.argtypes = [P, P]
        L.pe_expand_obs_codes.argtypes = [P, I32, I32, P, ctypes.c_int64, P, P, P, P, P]
    L.pe_get_info.argtypes = [P, P, P]
    L.pe_get_state.argtypes = [P, P, P, P, P, P]
    L.pe_set_state.argtypes = [P, P, P, P, P, P]
    L.pe_load_maps.argtypes = [P, I32, P, P, P, P, P]
    L.pe_synth_actions.argtypes = [P, U64, U32, P, P]
    L.pe_poll_errors.argtypes = [P, ctypes.POINTER(I32), P]
    L.pe_num_envs.argtypes = [P]
    L.pe_num_envs.restype = I32
    L.pe_kernel_variant.argtypes = [P]
    L.pe_kernel_variant.restype = I32
    L.pe_kernel_name.argtypes = [P]
    L.pe_prefetch_every.argtypes = [P]
    L.pe_prefetch_every.restype = I32
    L.pe_kernel_name.restype = ctypes.c_char_p
    L.pe_state_bytes.argtypes = [P]
    L.pe_state_bytes.restype = U64
    L.pe_last_error.argtypes = []
    L.pe_last_error.restype = ctypes.c_char_p
    D = ctypes.c_double
    L.pe_curriculum_enable.argtypes = [P, D, D, D, I32, I32, P]
    L.pe_curriculum_disable.argtypes = [P]
    L.pe_curriculum_get.argtypes = [P, P, P, P]
    L.pe_pystream_create.argtypes = [CP, ctypes.c_int64, ctypes.POINTER(P)]
    L.pe_pystream_next.argtypes = [P, I32, P, P]
    L.pe_pystream_getrandbits32.argtypes = [P]
    L.pe_pystream_getrandbits32.restype = U32
    L.pe_pystream_destroy.argtypes = [P]
    L.pe_mcts_create.argtypes = [P, I32, D, I32, ctypes.POINTER(P)]
    L.pe_mcts_destroy.argtypes = [P]
    L.pe_mcts_seed.argtypes = [P, P, U32, P]
    L.pe_mcts_set_rng.argtypes = [P, P, P]
    L.pe_mcts_get_rng.argtypes = [P, P, P]
    L.pe_mcts_search.argtypes = [P, P, P, P, P, P, P]
    for name in ("pe_create", "pe_destroy", "pe_seed", "pe_reset", "pe_step", "pe_get_info", "pe_get_state",
                 "pe_set_state", "pe_load_maps", "pe_synth_actions", "pe_poll_errors", "pe_pystream_create",
                 "pe_pystream_next", "pe_pystream_destroy", "pe_curriculum_enable", "pe_curriculum_disable",
                 "pe_curriculum_get", "pe_mcts_create", "pe_mcts_destroy", "pe_mcts_seed", "pe_mcts_set_rng",
                 "pe_mcts_get_rng", "pe_mcts_search", "pe_step_codes", "pe_obs_code_table",
                 "pe_expand_obs_codes"):
        if hasattr(L, name):
            getattr(L, name).restype = ctypes.c_int
    _lib = L
    return L


def check(rc, what):
    if rc != PE_OK:
        msg = lib().pe_last_error().decode(errors="replace")
        if rc == PE_ERR_ARG:
            raise ValueError(f"{what}: {msg}")
        if rc == PE_ERR_NOROOM:
            raise ValueError(f"{what}: {msg}")
        raise PlantOSNativeError(f"{what} failed ({rc}): {msg}")


def default_config(grid_size, num_plants, num_obstacles, lidar_range, lidar_channels):
    c = PEConfig()
    lib().pe_default_config(ctypes.byref(c), grid_size, num_plants, num_obstacles, lidar_range, lidar_channels)
    return c


class PyStream:
    """Host-side CPython `random` map stream (seed-exact reset layouts,
    plantos_env.py:338-372 after random.seed(seed)); see include/plantos_batch.h."""

    def __init__(self, grid_size, num_plants, num_obstacles, seed, thirsty_plant_prob=0.7,
                 map_generation_algo="original"):
        import numpy as np
        self._np = np
        self.G = grid_size
        c = default_config(grid_size, num_plants, num_obstacles, 1, 1)
        c.thirsty_plant_prob = float(thirsty_plant_prob)
        c.map_generation_algo = map_algo_id(map_generation_algo)
        h = ctypes.c_void_p()
        check(lib().pe_pystream_create(ctypes.byref(c), int(seed), ctypes.byref(h)), "pe_pystream_create")
        self._h = h

    def next(self, k):
        """next k maps in stream order: cells u8[k,G,G], rover i32[k,2] (numpy)."""
        np = self._np
        cells = np.zeros((k, self.G, self.G), np.uint8)
        rover = np.zeros((k, 2), np.int32)
        check(lib().pe_pystream_next(self._h, int(k), cells.ctypes.data_as(ctypes.c_void_p),
                                     rover.ctypes.data_as(ctypes.c_void_p)), "pe_pystream_next")
        return cells, rover

    def getrandbits32(self):
        return int(lib().pe_pystream_getrandbits32(self._h))

    def close(self):
        if getattr(self, "_h", None):
            lib().pe_pystream_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass
