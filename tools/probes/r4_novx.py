# Timing probe (wrong exact visit counts past 15; obs, rewards and the trajectory are
# unchanged): the overflow slot's writes (visit_bump_exact) removed from the step.
p = "rl-env_amd/csrc/pe_device.hpp"
s = open(p).read()
old = "  uint32_t* vp = st.vx + e * g.hstride + cell;\n  if (n == 14u) {"
assert s.count(old) == 1
s = s.replace(old, "  uint32_t* vp = st.vx + e * g.hstride + cell;\n  if (n == 99u) {")
old2 = "  } else if (n == 15u) {\n    atomicAdd(vp, 1u);"
assert s.count(old2) == 1
s = s.replace(old2, "  } else if (n == 98u) {\n    atomicAdd(vp, 1u);")
open(p, "w").write(s)
