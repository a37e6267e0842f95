#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ from the REFERENCE itself.

Runs only in the build container (the reference never travels to the GPU box).
The reference (`/root/reference/plantos_env.py` and its fork
`/root/reference/gradio-app/plantos_env_new.py`) is imported through the stub
shim in tools/refshim/ (gymnasium / pygame / viewer stand-ins).
Nothing from the reference is copied: only inputs and the reference's outputs
are written, as compressed numpy arrays (loadable with allow_pickle=False).

Fixtures written (all under tests/golden/):
  kat_seed0.npz          Appendix-B known-answer run (random.seed(0), 1000 steps)
  lidar_firsthit.npz     per-(C,R) first-hit maps derived from the reference's
                         _get_lidar_obs (plantos_env.py:260-292)
  maps_<cfg>.npz         consecutive reset() maps after random.seed(s)
                         (plantos_env.py:338-372, CPython `random` stream)
  inject_<cfg>.npz       state-injected single steps (fork semantics,
                         gradio-app/plantos_env_new.py:162-245) incl. pre-step obs
  traj_<cfg>.npz         DummyVecEnv-style multi-env rollouts with auto-reset
                         (A2C_training.py:216-218 semantics, SB3 step_wait)

Usage:  PYTHONDONTWRITEBYTECODE=1 python tools/gen_golden.py
"""
import hashlib
import os
import random
import sys
from collections import deque

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
OUT = os.path.join(REPO, "tests", "golden")
REF = "/root/reference"

sys.dont_write_bytecode = True
sys.path[:0] = [os.path.join(HERE, "refshim"), REF, os.path.join(REF, "gradio-app")]
import plantos_env  # noqa: E402  (reference, root env)
import plantos_env_new  # noqa: E402  (reference, gradio fork)

RootEnv = plantos_env.PlantOSEnv
ForkEnv = plantos_env_new.PlantOSEnvNew

# (name, grid, plants, obstacles, lidar_range, lidar_channels)
CONFIGS = {
    "g20": (20, 10, 12, 6, 16),      # BASELINE headline geometry
    "g21": (21, 8, 50, 2, 10),       # PlantOSEnv defaults (plantos_env.py:25-26)
    "g25": (25, 10, 12, 6, 16),      # A2C_training.py:206-212
    "g64": (64, 100, 120, 6, 64),    # stress geometry
    "g64r32": (64, 100, 120, 32, 64),
    "g7": (7, 3, 3, 3, 12),          # tiny grid: rays leave the map
    "g32": (32, 20, 30, 9, 24),
}

EMPTY, OBST, HYD, THIRSTY = 0, 1, 2, 3


def make(env_cls, cfg):
    G, P, O, R, C = CONFIGS[cfg]
    kw = dict(grid_size=G, num_plants=P, num_obstacles=O, lidar_range=R, lidar_channels=C)
    if env_cls is ForkEnv:
        kw["map_generation_algo"] = "original"
    return env_cls(**kw)


def cells_of(env):
    G = env.grid_size
    c = np.zeros((G, G), np.uint8)
    for (x, y) in env.obstacles:
        c[x, y] = OBST
    for (x, y), t in env.plants.items():
        c[x, y] = THIRSTY if t else HYD
    return c


def sha(obs):
    return hashlib.sha256(np.ascontiguousarray(obs, np.float32).tobytes()).digest()


# --------------------------------------------------------------------------- KAT
def gen_kat():
    G, P, O, R, C = CONFIGS["g20"]
    random.seed(0)
    env = make(ForkEnv, "g20")
    obs0, info0 = env.reset()
    cells0 = cells_of(env)
    rover0 = np.array(env.rover_pos, np.int32)
    plant_order = np.array(list(env.plants.keys()), np.int32)
    actions = np.random.default_rng(0).integers(0, 5, 1000).astype(np.int32)
    obs = [obs0]
    rew, term, trunc, rover, expl, coll = [], [], [], [], [], []
    for a in actions:
        o, r, te, tr, info = env.step(int(a))
        obs.append(o)
        rew.append(r)
        term.append(te)
        trunc.append(tr)
        rover.append(env.rover_pos)
        expl.append(info["explored_cells"])
        coll.append(info["total_collisions"])
    # the root env raises TypeError on watering a hydrated plant (plantos_env.py:217-220)
    random.seed(0)
    root = make(RootEnv, "g20")
    root.reset()
    raise_step = -1
    root_sum = 0.0
    for t, a in enumerate(actions):
        try:
            _, r, _, _, _ = root.step(int(a))
            root_sum += r
        except TypeError:
            raise_step = t
            break
    np.savez_compressed(
        os.path.join(OUT, "kat_seed0.npz"),
        config=np.array([G, P, O, R, C], np.int32),
        cells0=cells0, rover0=rover0, plant_order=plant_order,
        actions=actions, obs=np.array(obs, np.float32),
        reward=np.array(rew, np.float64), terminated=np.array(term, np.uint8),
        truncated=np.array(trunc, np.uint8), rover=np.array(rover, np.int32),
        explored=np.array(expl, np.int32), collisions=np.array(coll, np.int32),
        final_visits=env.visit_counts.astype(np.int32),
        final_explored=env.explored_map.astype(np.int8),
        root_raise_step=np.int32(raise_step), root_reward_sum=np.float64(root_sum),
        info0_total_cells=np.int32(info0["total_cells"]),
        reward_sum=np.float64(sum(rew)),
    )
    print("kat: sum", sum(rew), "root raises at", raise_step)


# ------------------------------------------------------------------ LIDAR probes
def gen_lidar_firsthit():
    """For each (C,R): place ONE obstacle at every cell of the (2R+1)^2 window
    around the rover and record, per ray, the distance the reference reports
    (0 = ray did not stop on it).  This pins the reference's int(r*cos),
    int(r*sin) offset table including the (0,0) and duplicate-cell quirks."""
    out = {}
    for (C, R) in [(16, 6), (10, 2), (64, 6), (64, 32), (12, 3), (24, 9), (8, 4), (5, 7), (3, 1)]:
        W = 2 * R + 1
        env = RootEnv(grid_size=W, num_plants=1, num_obstacles=0, lidar_range=R, lidar_channels=C)
        env.reset()
        env.plants = {}
        env.rover_pos = (R, R)
        env.visit_counts = np.zeros((W, W), np.int32)
        res = np.zeros((W * W, C), np.int16)
        for cx in range(W):
            for cy in range(W):
                env.obstacles = {(cx, cy)}
                o = env._get_lidar_obs()
                for i in range(C):
                    d = o[5 * i]
                    onehot = o[5 * i + 1:5 * i + 5]
                    if onehot[OBST] == 1.0:
                        res[cx * W + cy, i] = int(round(float(d) * R))
        out[f"C{C}_R{R}"] = res
    np.savez_compressed(os.path.join(OUT, "lidar_firsthit.npz"), **out)
    print("lidar first-hit maps:", list(out))


# --------------------------------------------------------------- reset streams
def gen_maps(cfg, seeds, resets):
    env = make(RootEnv, cfg)
    G = env.grid_size
    P = env.num_plants
    cells = np.zeros((len(seeds), resets, G, G), np.uint8)
    rover = np.zeros((len(seeds), resets, 2), np.int32)
    porder = np.zeros((len(seeds), resets, P, 2), np.int32)
    tail = np.zeros((len(seeds),), np.int64)
    obs0 = []
    for si, s in enumerate(seeds):
        random.seed(s)
        for k in range(resets):
            o, _ = env.reset()
            cells[si, k] = cells_of(env)
            rover[si, k] = env.rover_pos
            porder[si, k] = np.array(list(env.plants.keys()), np.int32)
            if k == 0:
                obs0.append(o)
        tail[si] = random.getrandbits(32)  # pins the exact number of MT draws consumed
    np.savez_compressed(
        os.path.join(OUT, f"maps_{cfg}.npz"), config=np.array(CONFIGS[cfg], np.int32),
        seeds=np.array(seeds, np.int64), cells=cells, rover=rover, plant_order=porder,
        next_u32=tail, obs0=np.array(obs0, np.float32))
    print(f"maps_{cfg}:", cells.shape)


# ------------------------------------------------------- state-injected steps
def random_state(rng, cfg, kind):
    G, P, O, R, C = CONFIGS[cfg]
    cells = np.zeros((G, G), np.uint8)
    dens = rng.choice([0.0, 0.03, 0.08, 0.2, 0.4])
    cells[rng.random((G, G)) < dens] = OBST
    free = np.argwhere(cells == 0)
    if len(free) < 2:
        cells[:] = 0
        free = np.argwhere(cells == 0)
    npl = int(rng.integers(0, min(P, len(free) - 1) + 1))
    pidx = rng.choice(len(free), size=npl, replace=False)
    for j in pidx:
        x, y = free[j]
        cells[x, y] = THIRSTY if rng.random() < 0.6 else HYD
    free_all = np.argwhere(cells != OBST)
    # rover placement: bias to borders and to plant cells
    u = rng.random()
    plants_at = np.argwhere((cells == HYD) | (cells == THIRSTY))
    if u < 0.25 and len(plants_at):
        rx, ry = plants_at[rng.integers(len(plants_at))]
    elif u < 0.5:
        border = [p for p in free_all if p[0] in (0, G - 1) or p[1] in (0, G - 1)]
        rx, ry = border[rng.integers(len(border))] if border else free_all[rng.integers(len(free_all))]
    else:
        rx, ry = free_all[rng.integers(len(free_all))]
    rx, ry = int(rx), int(ry)
    visits = np.zeros((G, G), np.int32)
    vm = rng.random((G, G)) < rng.choice([0.0, 0.2, 0.6, 0.95])
    vals = rng.geometric(rng.choice([0.5, 0.15, 0.05]), size=(G, G)).astype(np.int32)
    visits[vm] = vals[vm]
    visits[cells == OBST] = 0
    if rng.random() < 0.05:
        visits[rx, ry] = int(rng.choice([255, 256, 1000, 4000]))
    explored = np.zeros((G, G), np.int8)
    mode = rng.random()
    if mode < 0.6:
        explored[visits > 0] = 1       # bare-env invariant explored>0 <=> visit>0
    else:
        explored[(rng.random((G, G)) < 0.3) & (cells != OBST)] = 1  # curriculum-style divergence
    explored[rx, ry] = 2
    if rng.random() < 0.7:
        visits[rx, ry] = max(1, visits[rx, ry])
    step = int(rng.choice([0, 1, 5, 500, 998, 999, 1000, 1003]) if rng.random() < 0.5 else rng.integers(0, 1000))
    coll = int(rng.integers(0, 300))
    collided = bool(coll > 0 and rng.random() < 0.5)
    bonus = bool(rng.random() < 0.1)
    action = int(rng.integers(0, 5))
    if (cells[rx, ry] in (HYD, THIRSTY)) and rng.random() < 0.5:
        action = 4
    if kind == "complete":
        # everything explored except one free neighbour of the rover; move into it
        nbrs = []
        for a, (dx, dy) in enumerate([(-1, 0), (0, 1), (1, 0), (0, -1)]):
            nx, ny = rx + dx, ry + dy
            if 0 <= nx < G and 0 <= ny < G and cells[nx, ny] != OBST:
                nbrs.append((a, nx, ny))
        if nbrs:
            a, nx, ny = nbrs[rng.integers(len(nbrs))]
            explored[:] = 0
            explored[cells != OBST] = 1
            explored[rx, ry] = 2
            explored[nx, ny] = 0
            if rng.random() < 0.5:
                visits[nx, ny] = 0
            action = a
            bonus = bool(rng.random() < 0.2)
    return dict(cells=cells, visits=visits, explored=explored, rover=(rx, ry), step=step,
                coll=coll, collided=collided, bonus=bonus, action=action)


def inject(env, st):
    G = env.grid_size
    c = st["cells"]
    env.obstacles = set((int(x), int(y)) for x, y in np.argwhere(c == OBST))
    env.plants = {}
    for x in range(G):
        for y in range(G):
            if c[x, y] in (HYD, THIRSTY):
                env.plants[(x, y)] = bool(c[x, y] == THIRSTY)
    env.rover_pos = st["rover"]
    env.visit_counts = st["visits"].copy()
    env.explored_map = st["explored"].copy()
    env.step_count = st["step"]
    env.total_collisions = st["coll"]
    env.collided_with_wall = st["collided"]
    env.completion_bonus_given = st["bonus"]


def gen_inject(cfg, n, seed):
    G, P, O, R, C = CONFIGS[cfg]
    rng = np.random.default_rng(seed)
    env = make(ForkEnv, cfg)
    random.seed(seed)
    env.reset()
    A = {k: [] for k in ["cells", "visits", "explored", "scal", "action", "obs_pre", "obs",
                         "reward", "term", "trunc", "cells_post", "visits_post", "explored_post",
                         "scal_post", "root_raises"]}
    for i in range(n):
        st = random_state(rng, cfg, "complete" if i % 10 == 9 else "random")
        inject(env, st)
        obs_pre = env._get_obs()
        a = st["action"]
        root_raises = bool(a == 4 and st["cells"][st["rover"]] == HYD)
        o, r, te, tr, info = env.step(a)
        A["cells"].append(st["cells"])
        A["visits"].append(st["visits"])
        A["explored"].append(st["explored"])
        A["scal"].append([st["rover"][0], st["rover"][1], st["step"], st["coll"], int(st["collided"]), int(st["bonus"])])
        A["action"].append(a)
        A["obs_pre"].append(obs_pre)
        A["obs"].append(o)
        A["reward"].append(r)
        A["term"].append(te)
        A["trunc"].append(tr)
        A["cells_post"].append(cells_of(env))
        A["visits_post"].append(env.visit_counts.copy())
        A["explored_post"].append(env.explored_map.copy())
        A["scal_post"].append([env.rover_pos[0], env.rover_pos[1], env.step_count, env.total_collisions,
                               int(env.collided_with_wall), int(env.completion_bonus_given),
                               int(info["explored_cells"]), int(info["total_cells"]),
                               int(info["thirsty_plants"]), int(info["hydrated_plants"])])
        A["root_raises"].append(root_raises)
    vdt = np.uint16 if G > 32 else np.int32
    np.savez_compressed(
        os.path.join(OUT, f"inject_{cfg}.npz"), config=np.array(CONFIGS[cfg], np.int32),
        cells=np.array(A["cells"], np.uint8), visits=np.array(A["visits"], vdt),
        explored=np.array(A["explored"], np.int8), scal=np.array(A["scal"], np.int32),
        action=np.array(A["action"], np.int32), obs_pre=np.array(A["obs_pre"], np.float32),
        obs=np.array(A["obs"], np.float32), reward=np.array(A["reward"], np.float64),
        term=np.array(A["term"], np.uint8), trunc=np.array(A["trunc"], np.uint8),
        cells_post=np.array(A["cells_post"], np.uint8), visits_post=np.array(A["visits_post"], vdt),
        explored_post=np.array(A["explored_post"], np.int8), scal_post=np.array(A["scal_post"], np.int32),
        root_raises=np.array(A["root_raises"], np.uint8))
    print(f"inject_{cfg}: {n} cases, term={int(np.sum(A['term']))}")


# ------------------------------------------------ multi-env rollouts (auto-reset)
def bfs_action(env):
    """Heuristic explorer (part of the INPUT generation, not of the reference):
    move toward the nearest never-visited free cell."""
    G = env.grid_size
    sx, sy = env.rover_pos
    if env.visit_counts[sx, sy] == 0:
        pass
    prev = {(sx, sy): None}
    q = deque([(sx, sy)])
    target = None
    while q:
        x, y = q.popleft()
        if env.explored_map[x, y] == 0:
            target = (x, y)
            break
        for dx, dy in [(-1, 0), (0, 1), (1, 0), (0, -1)]:
            nx, ny = x + dx, y + dy
            if 0 <= nx < G and 0 <= ny < G and (nx, ny) not in env.obstacles and (nx, ny) not in prev:
                prev[(nx, ny)] = (x, y)
                q.append((nx, ny))
    if target is None:
        return 4
    cur = target
    while prev[cur] != (sx, sy):
        cur = prev[cur]
    d = (cur[0] - sx, cur[1] - sy)
    return [(-1, 0), (0, 1), (1, 0), (0, -1)].index(d)


def gen_traj(cfg, n_envs, steps, seed, policy):
    """DummyVecEnv semantics: envs reset in index order, stepped in index order;
    on terminated|truncated: terminal obs kept, env.reset() (global `random`
    stream), returned obs is the reset obs."""
    envs = [make(ForkEnv, cfg) for _ in range(n_envs)]
    G = envs[0].grid_size
    random.seed(seed)
    rng = np.random.default_rng(seed + 1000)
    obs0 = np.array([e.reset()[0] for e in envs], np.float32)
    maps0 = np.array([cells_of(e) for e in envs], np.uint8)
    rov0 = np.array([e.rover_pos for e in envs], np.int32)
    D = obs0.shape[1]
    acts = np.zeros((steps, n_envs), np.int32)
    obs = np.zeros((steps, n_envs, D), np.float32)
    term_obs = np.zeros((steps, n_envs, D), np.float32)
    rew = np.zeros((steps, n_envs), np.float64)
    te = np.zeros((steps, n_envs), np.uint8)
    tr = np.zeros((steps, n_envs), np.uint8)
    reset_maps = []
    for t in range(steps):
        for i, e in enumerate(envs):
            if policy == "random":
                a = int(rng.integers(0, 5))
            else:  # mostly-greedy explorer with some noise (finishes episodes)
                a = bfs_action(e) if rng.random() < 0.9 else int(rng.integers(0, 5))
            acts[t, i] = a
            o, r, a_te, a_tr, _ = e.step(a)
            rew[t, i] = r
            te[t, i] = a_te
            tr[t, i] = a_tr
            if a_te or a_tr:
                term_obs[t, i] = o
                o, _ = e.reset()
                reset_maps.append((t, i, cells_of(e), e.rover_pos))
            obs[t, i] = o
    np.savez_compressed(
        os.path.join(OUT, f"traj_{cfg}_{policy}.npz"), config=np.array(CONFIGS[cfg], np.int32),
        seed=np.int64(seed), maps0=maps0, rover0=rov0, obs0=obs0, actions=acts, obs=obs,
        terminal_obs=term_obs, reward=rew, terminated=te, truncated=tr,
        reset_t=np.array([m[0] for m in reset_maps], np.int32),
        reset_env=np.array([m[1] for m in reset_maps], np.int32),
        reset_cells=np.array([m[2] for m in reset_maps], np.uint8).reshape(-1, G, G),
        reset_rover=np.array([m[3] for m in reset_maps], np.int32).reshape(-1, 2),
        next_u32=np.int64(random.getrandbits(32)))
    print(f"traj_{cfg}_{policy}: {n_envs}x{steps}, resets={len(reset_maps)}, term={int(te.sum())}")


def load_curriculum_wrapper(source="A2C_training.py"):
    """The reference's own CurriculumWrapper class (A2C_training.py:37-109, or the
    trainingCode.py:24-98 variant), compiled from the reference file: only that class
    definition is executed (the module's stable_baselines3 / sb3_contrib / matplotlib
    imports and directory creation are skipped -- those packages are absent here and
    not part of the wrapper)."""
    import ast
    import gymnasium as gym_shim
    path = os.path.join(REF, source)
    tree = ast.parse(open(path).read())
    node = next(n for n in tree.body if isinstance(n, ast.ClassDef) and n.name == "CurriculumWrapper")
    ns = {"gym": gym_shim, "np": np}
    exec(compile(ast.Module(body=[node], type_ignores=[]), path, "exec"), ns)  # noqa: S102
    return ns["CurriculumWrapper"]


def gen_curriculum(cfg, n_envs, steps, seed, policy, variant="a2c"):
    """DummyVecEnv over CurriculumWrapper(fork env, 40, 100) (A2C_training.py:114-126
    with use_curriculum=True; Monitor omitted: it does not change the step data), or
    (variant "tc") over trainingCode.py's CurriculumWrapper(env, 30, 100) as its
    make_env_wrapper builds it (trainingCode.py:103-111)."""
    if variant == "tc":
        CW = load_curriculum_wrapper("trainingCode.py")
        envs = [CW(make(ForkEnv, cfg), initial_threshold=30.0, max_threshold=100.0) for _ in range(n_envs)]
    else:
        CW = load_curriculum_wrapper()
        envs = [CW(make(ForkEnv, cfg), initial_threshold=40.0, max_threshold=100.0) for _ in range(n_envs)]
    G = envs[0].env.grid_size
    random.seed(seed)
    np.random.seed(seed + 7)  # the wrapper's np.random.randint "maze seeds" (ignored by the env)
    rng = np.random.default_rng(seed + 1000)
    obs0 = np.array([w.reset()[0] for w in envs], np.float32)
    D = obs0.shape[1]
    acts = np.zeros((steps, n_envs), np.int32)
    obs = np.zeros((steps, n_envs, D), np.float32)
    term_obs = np.zeros((steps, n_envs, D), np.float32)
    rew = np.zeros((steps, n_envs), np.float64)
    te = np.zeros((steps, n_envs), np.uint8)
    tr = np.zeros((steps, n_envs), np.uint8)
    thr = np.zeros((steps, n_envs), np.float64)
    visits_sum = np.zeros((steps, n_envs), np.int64)
    for t in range(steps):
        for i, w in enumerate(envs):
            if policy == "random":
                a = int(rng.integers(0, 5))
            else:
                a = bfs_action(w.env) if rng.random() < 0.9 else int(rng.integers(0, 5))
            acts[t, i] = a
            o, r, a_te, a_tr, _ = w.step(a)
            rew[t, i] = r
            te[t, i] = a_te
            tr[t, i] = a_tr
            if a_te or a_tr:
                term_obs[t, i] = o
                o, _ = w.reset()
            obs[t, i] = o
            thr[t, i] = w.exploration_threshold
            visits_sum[t, i] = int(w.env.visit_counts.sum())
    fin = np.array([[w.episode_count, w.successful_explorations, w.episodes_on_current_maze,
                     int(w.maze_completed) | (2 * int(w.persistent_visit_counts is not None))] for w in envs],
                   np.int32)
    name = f"curriculum_{'tc_' if variant == 'tc' else ''}{cfg}_{policy}"
    np.savez_compressed(
        os.path.join(OUT, f"{name}.npz"), config=np.array(CONFIGS[cfg], np.int32),
        seed=np.int64(seed), obs0=obs0, actions=acts, obs=obs, terminal_obs=term_obs, reward=rew,
        terminated=te, truncated=tr, threshold=thr, visits_sum=visits_sum, final_counters=fin,
        next_u32=np.int64(random.getrandbits(32)))
    print(f"{name}: {n_envs}x{steps}, term={int(te.sum())}, thr_max={thr.max()}, G={G}, "
          f"successes={fin[:, 1].tolist()}")


def load_mcts():
    """The reference's MCTS module (mcts_custom_trainer.py), imported through the shim.
    Its sim envs are built from the module-level name `PlantOSEnv` (:227-233); that name
    is pointed at the fork env, whose watering of a hydrated plant returns R_MISTAKE
    (gradio-app/plantos_env_new.py:236-245) -- with the root env a random rollout that
    waters a hydrated plant raises TypeError (plantos_env.py:217-220) and aborts the
    search.  best_action (:62-69) is wrapped to RECORD the root's children (action,
    visits, value in insertion order); the returned action is the reference's own."""
    import mcts_custom_trainer as M
    M.PlantOSEnv = ForkEnv
    rec = []
    orig = M.MCTSNode.best_action

    def best_action(self):
        if self.parent is None:
            rec.append([(a, c.visits, c.value) for a, c in self.children.items()])
        return orig(self)

    M.MCTSNode.best_action = best_action
    return M, rec


def np_state_crc(st):
    import zlib
    return zlib.crc32(np.ascontiguousarray(st[1], np.uint32).tobytes())


def gen_mcts(name, cfg, n_sims, max_depth, chains, decisions, seed, inject_cases=0, c_param=1.414):
    """MCTS.search (mcts_custom_trainer.py:91-139) decisions of the reference.

    chains: episodes from reset (random.seed(seed+k) map, np.random.seed(seed+100+k)
    stream), `decisions` searches each, the real env stepped with the chosen action
    between them (train_mcts, :298-302).  inject_cases: single searches from
    injected states (step counts near max_steps, nearly explored maps), each with
    its own np.random.seed."""
    M, rec = load_mcts()
    G = CONFIGS[cfg][0]
    A = {k: [] for k in ["chain", "cseed", "cells", "visits", "explored", "scal", "action", "order",
                         "cvisits", "cvalue", "pos_out", "crc_out"]}

    def one(env, mcts, chain, cseed):
        A["chain"].append(chain)
        A["cseed"].append(cseed)
        A["cells"].append(cells_of(env))
        A["visits"].append(env.visit_counts.astype(np.int32).copy())
        A["explored"].append(env.explored_map.astype(np.int8).copy())
        A["scal"].append([env.rover_pos[0], env.rover_pos[1], env.step_count, env.total_collisions,
                          int(env.collided_with_wall), int(env.completion_bonus_given)])
        rec.clear()
        a = mcts.search(None)
        kids = rec[0]
        order = np.full(5, -1, np.int32)
        cv = np.zeros(5, np.int32)
        cval = np.zeros(5, np.float64)
        for j, (ca, vis, val) in enumerate(kids):
            order[j], cv[j], cval[j] = ca, vis, val
        A["action"].append(a)
        A["order"].append(order)
        A["cvisits"].append(cv)
        A["cvalue"].append(cval)
        st = np.random.get_state()
        A["pos_out"].append(st[2])
        A["crc_out"].append(np_state_crc(st))
        return a

    nterm = 0
    for k in range(chains):
        env = make(ForkEnv, cfg)
        random.seed(seed + k)
        env.reset()
        np.random.seed(seed + 100 + k)
        mcts = M.MCTS(env, n_simulations=n_sims, c_param=c_param, max_depth=max_depth)
        for d in range(decisions):
            a = one(env, mcts, k, seed + 100 + k if d == 0 else -1)
            _, _, te, tr, _ = env.step(int(a))
            if te or tr:
                nterm += 1
                break
    rng = np.random.default_rng(seed + 7)
    for i in range(inject_cases):
        env = make(ForkEnv, cfg)
        random.seed(seed + 1000 + i)
        env.reset()
        st = random_state(rng, cfg, "complete" if i % 3 == 2 else "random")
        if i % 4 == 1:
            st["step"] = int(rng.choice([995, 998, 999, 1000, 1004]))
        inject(env, st)
        np.random.seed(seed + 2000 + i)
        mcts = M.MCTS(env, n_simulations=n_sims, c_param=c_param, max_depth=max_depth)
        one(env, mcts, chains + i, seed + 2000 + i)
    np.savez_compressed(
        os.path.join(OUT, f"mcts_{name}.npz"), config=np.array(CONFIGS[cfg], np.int32),
        n_sims=np.int32(n_sims), max_depth=np.int32(max_depth), c_param=np.float64(c_param),
        chain=np.array(A["chain"], np.int32), cseed=np.array(A["cseed"], np.int64),
        cells=np.array(A["cells"], np.uint8).reshape(-1, G, G),
        visits=np.array(A["visits"], np.int32).reshape(-1, G, G),
        explored=np.array(A["explored"], np.int8).reshape(-1, G, G),
        scal=np.array(A["scal"], np.int32).reshape(-1, 6), action=np.array(A["action"], np.int32),
        order=np.array(A["order"], np.int32).reshape(-1, 5), cvisits=np.array(A["cvisits"], np.int32).reshape(-1, 5),
        cvalue=np.array(A["cvalue"], np.float64).reshape(-1, 5), pos_out=np.array(A["pos_out"], np.int32),
        crc_out=np.array(A["crc_out"], np.uint32))
    print(f"mcts_{name}: {len(A['action'])} searches, episodes ended={nterm}")


def main():
    os.makedirs(OUT, exist_ok=True)
    gen_kat()
    gen_lidar_firsthit()
    gen_maps("g20", [0, 1, 2, 3, 7, 42, 123, 2024], 6)
    gen_maps("g21", [0, 1, 5], 4)
    gen_maps("g25", [0, 3], 4)
    gen_maps("g64", [0, 9], 3)
    gen_maps("g7", [0, 1, 2, 3], 6)
    gen_maps("g32", [11], 3)
    gen_inject("g20", 3000, 1)
    gen_inject("g21", 500, 2)
    gen_inject("g25", 500, 3)
    gen_inject("g64", 120, 4)
    gen_inject("g64r32", 80, 5)
    gen_inject("g7", 400, 6)
    gen_inject("g32", 200, 7)
    gen_traj("g20", 4, 1100, 0, "random")
    gen_traj("g20", 3, 900, 5, "explore")
    gen_traj("g7", 4, 300, 3, "explore")
    gen_traj("g21", 2, 400, 8, "explore")
    gen_curriculum("g20", 4, 1500, 11, "explore")
    gen_curriculum("g7", 6, 400, 12, "explore")
    gen_curriculum("g20", 3, 2100, 13, "random")


def gen_maze_maps(name, cfgt, seeds, resets):
    """Consecutive reset() layouts of the fork with map_generation_algo='maze'
    (gradio-app/plantos_env_new.py:408-604: DFS maze on a (G-1)//6 meta grid,
    irregular rooms, path bulges; falls back to the original generator when the
    maze has no room for the plants + rover)."""
    G, P, O, R, C = cfgt
    env = ForkEnv(grid_size=G, num_plants=P, num_obstacles=O, lidar_range=R, lidar_channels=C,
                  map_generation_algo="maze")
    cells = np.zeros((len(seeds), resets, G, G), np.uint8)
    rover = np.zeros((len(seeds), resets, 2), np.int32)
    porder = np.zeros((len(seeds), resets, P, 2), np.int32)
    tail = np.zeros((len(seeds),), np.int64)
    obs0 = []
    import contextlib
    import io
    for si, s in enumerate(seeds):
        random.seed(s)
        for k in range(resets):
            with contextlib.redirect_stdout(io.StringIO()):  # the fallback prints a warning
                o, _ = env.reset()
            cells[si, k] = cells_of(env)
            rover[si, k] = env.rover_pos
            porder[si, k] = np.array(list(env.plants.keys()), np.int32).reshape(P, 2)
            if k == 0:
                obs0.append(o)
        tail[si] = random.getrandbits(32)
    np.savez_compressed(
        os.path.join(OUT, f"maze_{name}.npz"), config=np.array(cfgt, np.int32),
        seeds=np.array(seeds, np.int64), cells=cells, rover=rover, plant_order=porder,
        next_u32=tail, obs0=np.array(obs0, np.float32))
    free = (cells != OBST).reshape(len(seeds) * resets, -1).sum(1)
    print(f"maze_{name}:", cells.shape, "free cells min/max", free.min(), free.max())


def main_maze():
    os.makedirs(OUT, exist_ok=True)
    gen_maze_maps("g20", (20, 10, 12, 6, 16), [0, 1, 2, 3, 7, 42], 5)
    gen_maze_maps("g25", (25, 10, 12, 6, 16), [0, 5, 11], 4)
    gen_maze_maps("g13", (13, 5, 6, 3, 12), [0, 1, 2], 5)
    gen_maze_maps("g7", (7, 3, 3, 3, 12), [0, 1, 2, 3], 6)
    gen_maze_maps("g32", (32, 20, 30, 9, 24), [4, 9], 3)
    gen_maze_maps("g64", (64, 100, 120, 6, 64), [0, 9], 2)
    gen_maze_maps("g7fallback", (7, 30, 3, 3, 12), [0, 1, 2], 4)
    gen_maze_maps("g19", (19, 120, 12, 6, 16), [3, 4], 3)


def main_mcts():
    os.makedirs(OUT, exist_ok=True)
    gen_mcts("g7", "g7", 30, 40, 4, 40, 500, inject_cases=30)
    gen_mcts("g20", "g20", 50, 100, 3, 12, 600, inject_cases=24)
    gen_mcts("g25", "g25", 50, 100, 1, 8, 700)
    gen_mcts("g20d", "g20", 100, 50, 1, 4, 800)


def main_curriculum_tc():
    """trainingCode.py's CurriculumWrapper (threshold marks the maze completed
    without terminating)."""
    os.makedirs(OUT, exist_ok=True)
    gen_curriculum("g20", 3, 2100, 21, "random", "tc")
    gen_curriculum("g7", 6, 500, 22, "explore", "tc")
    gen_curriculum("g20", 4, 1500, 23, "explore", "tc")


if __name__ == "__main__":
    if sys.argv[1:] == ["curriculum_tc"]:
        main_curriculum_tc()
    elif sys.argv[1:] == ["mcts"]:
        main_mcts()
    elif sys.argv[1:] == ["maze"]:
        main_maze()
    else:
        main()
