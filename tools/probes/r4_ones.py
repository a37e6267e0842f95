# Timing probe (wrong results), the control of r4_noround2b.py: the real dependent
# round 2, the LDS visit rows forced to a visit count of 1 in every cell.
p = "rl-env_amd/csrc/plantos_batch.hip"
s = open(p).read()
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
