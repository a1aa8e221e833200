import sys, time
sys.path.insert(0, ".")
from orb_slam2_with_comment_amd import synth_map as SM
from orb_slam2_with_comment_amd.optimizer import LocalBA
problem, _ = SM.local_ba_problem(seed=42)
ba = LocalBA(0)
for _ in range(5): ba.run(problem)
t0=time.perf_counter()
for _ in range(10): r = ba.run(problem)
print("per call us", (time.perf_counter()-t0)/10*1e6, r["iterations"], flush=True)
