# Timing probe (wrong exact counts): the overflow slot's no-return atomic add
# (visit_bump_exact, n == 15) as a plain store -- what the atomics cost the step.
p = "rl-env_amd/csrc/pe_device.hpp"
s = open(p).read()
old = "    atomicAdd(vp, 1u);  // no-return atomic: the count is never read by a step"
assert s.count(old) == 1
s = s.replace(old, "    *vp = 16u;")
open(p, "w").write(s)
