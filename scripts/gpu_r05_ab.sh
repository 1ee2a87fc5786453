# Round 5 A/B of builds or options: variants in $VARIANTS, each
# "name:lib_dir:ENV=V,ENV2=V2" (lib_dir "-" = the tree's lib; env optional),
# run on the configs in $CFGS (s8, c2, c5, c3; default s8), alternated $REPS
# times (default 2).  Prints GCUPS and ms per step of the default and the
# reference scoring.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r05ab}
mkdir -p $O
for rep in $(seq 1 ${REPS:-2}); do
  for vv in $VARIANTS; do
    name=${vv%%:*}; rest=${vv#*:}; libd=${rest%%:*}; envs=${rest#*:}; [ "$envs" = "$rest" ] && envs=""
    lib=ece1782-smith-waterman-cuda_amd/lib/libswamd.so
    [ "$libd" != "-" ] && lib=ece1782-smith-waterman-cuda_amd/$libd/libswamd.so
    for c in ${CFGS:-s8}; do
      case $c in s8) args="--shard-of 8" ;; s4) args="--shard-of 4" ;; s2) args="--shard-of 2" ;; c2) args="" ;; c5) args="--config c5" ;; c3) args="--config c3" ;; *) echo "unknown config $c"; exit 1 ;; esac
      env SW_AMD_LIB=$lib ${envs//,/ } timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-verify --sustained-seconds 0 $args ${BARGS} > $O/${c}_${name}_$rep.json 2> $O/${c}_${name}_$rep.err || { echo "$c $name FAILED"; tail -20 $O/${c}_${name}_$rep.err; exit 1; }
      python3 -c "
import json
d=json.loads(open('$O/${c}_${name}_$rep.json').read().strip().split(chr(10))[-1]); r=d.get('reference_scoring',{})
print('$c $name $rep', d['value'], d['ms_per_step'], r.get('value'), r.get('ms_per_step'), d['kernels']['inter'])"
    done
  done
done
echo RC=0
