# What the guard bands flag per query of C3 (SW_RESCUE_STATS, one step).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/rstats
mkdir -p $O
SW_RESCUE_STATS=1 timeout -k 10 600 python3 bench.py --config c3 --no-cpu-baseline --steps 1 --warmup 0 > $O/c3.json 2> $O/c3.err
rc=$?; echo RC=$rc; grep "rescue:" $O/c3.err | grep "ge 2" | cut -c1-230; exit $rc
