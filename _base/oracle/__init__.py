"""
CPU oracle for the swarm rollout hot path -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and the cpu_baseline leg of bench.py
may import this package, and only as the checker or the timed CPU
comparator.  The product (swarmrl_amd/) never imports, links or runs it.

  swarm_oracle.c  C restatement of BD + WCA + steepest descent + vision cone
                  + field distances in the shared number formats
  oracle.py       ctypes wrapper
  refsem.py       numpy restatement of the reference's semantics (schedule,
                  placement, signed angle, vision cones, field tasks)
"""
