# Timing probe (wrong results): the one-word sector kernel's visit-row loads made
# independent of the loader env's position (fixed rows 0..6 of slot 0), so that hipcc
# issues them with round 1 -- what the step costs with no dependent second round.
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
assert old in s
s = s.replace(old, new)
open(p, "w").write(s)
