"""Byte codes of the observation (include/plantos_batch.h pe_config.obs_codes).

Every obs value of PlantOSEnv._get_lidar_obs (plantos_env.py:251-315) is one of
fewer than 256 table floats: a LIDAR distance float(r / R) (288), a one-hot 0.0 /
1.0 (289-292), a position float(x / G) (295-296) or a visit value
float(min(v, 10) / 10) (308).  The step kernels' byte-coded tile holds one byte per
value (pe_coop.hpp ObsW<uint8_t>):

    code r (0..R)   -> float(r / R)        code R + 1      -> 1.0
    code 80 + v     -> float(min(v,10)/10)  code 96 + x     -> float(x / G)

so a sharded job can move 5C+27 bytes per env across the host boundary instead of
4(5C+27) and expand them once on the consumer's side (pe_expand_obs_codes).  This
module is the host side of that format: the table (the same f32 quotients as
pe_obs_code_table), an encoder for f32 obs rows, and a host expansion.
"""
import numpy as np

CODE_VIS, CODE_POS = 80, 96  # pe_coop.hpp kCodeVis / kCodePos


def code_table(grid_size, lidar_range):
    """float32[256]: the value of every code (unused codes 0.0)."""
    G, R = int(grid_size), int(lidar_range)
    t = np.zeros(256, np.float32)
    for c in range(256):
        if c <= R:
            t[c] = np.float32(c / R)
        elif c == R + 1:
            t[c] = np.float32(1.0)
        elif CODE_VIS <= c < CODE_VIS + 16:
            t[c] = np.float32(min(c - CODE_VIS, 10) / 10.0)
        elif CODE_POS <= c < CODE_POS + G:
            t[c] = np.float32((c - CODE_POS) / G)
    return t


def encode_obs(obs, grid_size, lidar_channels, lidar_range):
    """u8 codes of f32 obs rows [..., 5C+27] (column meaning as _get_lidar_obs lays
    them out); expand(encode(x)) == x bit for bit for every obs the env produces."""
    obs = np.asarray(obs, np.float32)
    C, R, G = int(lidar_channels), int(lidar_range), int(grid_size)
    out = np.zeros(obs.shape, np.uint8)
    lid = obs[..., :5 * C].reshape(obs.shape[:-1] + (C, 5))
    o = out[..., :5 * C].reshape(out.shape[:-1] + (C, 5))
    o[..., 0] = np.rint(lid[..., 0].astype(np.float64) * R).astype(np.uint8)        # distance r
    o[..., 1:] = np.where(lid[..., 1:] != 0.0, R + 1, 0).astype(np.uint8)           # one-hot
    out[..., :5 * C] = o.reshape(out[..., :5 * C].shape)
    out[..., 5 * C:5 * C + 2] = (CODE_POS + np.rint(obs[..., 5 * C:5 * C + 2].astype(np.float64) * G)).astype(np.uint8)
    out[..., 5 * C + 2:] = (CODE_VIS + np.rint(obs[..., 5 * C + 2:].astype(np.float64) * 10)).astype(np.uint8)
    return out


def io_layout(n, obs_dim):
    """Byte offsets of one code-mode io buffer: codes u8 [n, D] | (to 16 B) reward f32
    [n] | terminated u8 [n] | truncated u8 [n] | (to 16 B); returns (reward_off,
    term_off, trunc_off, total) -- total a multiple of 16, so buffers laid back to back
    (a gather's) keep every block 16-B aligned."""
    ro = (n * obs_dim + 15) & ~15
    return ro, ro + 4 * n, ro + 5 * n, (ro + 6 * n + 15) & ~15


def expand_host(src, blocks, rows, obs_dim, stride, table, obs, reward=None, terminated=None, truncated=None):
    """Host twin of pe_expand_obs_codes (CPU tensors / arrays): block b of `src` (u8,
    flat) at b * stride -> rows [b*rows, (b+1)*rows) of the outputs."""
    src = np.asarray(src).reshape(-1)
    ro, to, tro, _ = io_layout(rows, obs_dim)
    nd = rows * obs_dim
    for b in range(blocks):
        base = b * stride
        obs[b * rows:(b + 1) * rows] = table[src[base:base + nd]].reshape(rows, obs_dim)
        if reward is not None:
            reward[b * rows:(b + 1) * rows] = src[base + ro:base + to].view(np.float32)
        if terminated is not None:
            terminated[b * rows:(b + 1) * rows] = src[base + to:base + tro]
        if truncated is not None:
            truncated[b * rows:(b + 1) * rows] = src[base + tro:base + tro + rows]
