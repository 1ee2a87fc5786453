# Round 4 sweep: the 1/8 share (or $CFG) under environment overrides, one
# bench line each, alternated twice (REF=1: with the reference scoring).  SWEEP="name:VAR=v,VAR2=w name2:..."
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r04sweep}
mkdir -p $O
RFLAG=--no-reference-scoring
[ -n "$REF" ] && RFLAG=
for rep in 1 2; do
  for item in ${SWEEP:-base:X=1}; do
    name=${item%%:*}; envs=${item#*:}
    env $(echo $envs | tr ',' ' ') timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-verify --sustained-seconds 0 $RFLAG ${CFG:---shard-of 8} > $O/${name}_$rep.json 2> $O/${name}_$rep.err || { echo "$name FAILED"; tail -20 $O/${name}_$rep.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('$O/${name}_$rep.json').read().strip().split(chr(10))[-1])
r=d.get('reference_scoring',{})
print('$name', $rep, d['value'], d['ms_per_step'], d.get('kernel_ms_per_scan',{}).get('scan_total'), r.get('value'), r.get('ms_per_step'))"
  done
done
