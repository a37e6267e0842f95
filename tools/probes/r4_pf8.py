# A/B variant: the prefetch kernel at 8 waves per SIMD (<= 64 VGPRs) instead of the
# 6 its 84 VGPRs allow -- more maps in flight per launch.
p = "rl-env_amd/csrc/plantos_batch.hip"
s = open(p).read()
old = "__global__ __launch_bounds__(256) void pe_prefetch_kernel(StepArgs a, int all) {"
assert s.count(old) == 1
s = s.replace(old, "__global__ __launch_bounds__(256, 8) void pe_prefetch_kernel(StepArgs a, int all) {")
open(p, "w").write(s)
