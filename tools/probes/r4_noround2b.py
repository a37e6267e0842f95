# Timing probe (wrong results): as r4_noround2.py (visit-row loads independent of the
# position, so hipcc issues them with round 1), and the LDS visit rows forced to a
# visit count of 1 in every cell (the loaded bits kept live through an OR of bit 0),
# so that no env explores or terminates: the same resets as the real kernel.
p = "rl-env_amd/csrc/plantos_batch.hip"
s = open(p).read()
old = """      const uint32_t* lvb = vis_env(st, g, el, lw.w);  // (lw.w: the loader env's episode)
      {
#pragma unroll
        for (int j = 0; j < JV; ++j) {
          const int kk = sub + LT * j;
          const int xr = lx - 3 + kk;"""
new = """      const uint32_t* lvb = vis_env(st, g, el, 0u);
      {
#pragma unroll
        for (int j = 0; j < JV; ++j) {
          const int kk = sub + LT * j;
          const int xr = kk;"""
assert s.count(old) == 1
s = s.replace(old, new)
old2 = """          lvis[k * LS + le] = vo ? ((lo >> vo) | (hi << (32 - vo))) : lo;
        }
      }
    } else {"""
new2 = """          lvis[k * LS + le] = 0x11111111u | (((vo ? ((lo >> vo) | (hi << (32 - vo))) : lo)) & 1u);
        }
      }
    } else {"""
assert s.count(old2) == 1
s = s.replace(old2, new2)
open(p, "w").write(s)
