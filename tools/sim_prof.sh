#!/bin/bash
# rocprofv3 kernel stats of the simulated N-rank per-rank search step (tools/sim_dist.py)
set -u
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p $R/gpurun_out
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_sim -o run --output-format csv -- \
  python3 $R/tools/sim_dist.py --world ${WORLD:-8} --steps 20 > $R/gpurun_out/prof_sim.log 2>&1
rc=$?
tail -1 $R/gpurun_out/prof_sim.log
python3 - <<PY
import csv, glob
f = glob.glob("$R/gpurun_out/prof_sim/**/run_kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
# last 20 steps x the kernels of one step: print the tail of the trace (timed region)
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
tail = rows[-40:]
t0 = int(tail[0]["Start_Timestamp"])
for r in tail:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f'{(s - t0)/1e3:9.1f} {(e - s)/1e3:8.1f}us  grid={r["Grid_Size_X"]:>8s} {r["Kernel_Name"][:90]}')
PY
exit $rc
