# Timing probe (wrong obs): the 5x5 visit slice written as one constant table value
# (every lane reads tvis[1]) -- whether the slice's data-dependent LDS reads / values
# cost the step anything.
p = "rl-env_amd/csrc/pe_quad.hpp"
s = open(p).read()
old = "    for (int ly = 0; ly < 5; ++ly) t[ly] = tvis[(v >> (4 * ly)) & 15u];"
assert s.count(old) == 1
s = s.replace(old, "    for (int ly = 0; ly < 5; ++ly) t[ly] = tvis[((v >> (4 * ly)) & 15u) ? 1u : 1u];")
open(p, "w").write(s)
