# Round 4 A/B on C5, after the GPU suite: the standalone intra launch at
# 20 / 16 rows per lane in 12-wave workgroups (one per CU) with the LDS
# conveyor (default build), at 10 in 4-wave ones with it, and (lib/ab4, built
# with IX2FLAGS="-DSW_IX2_WIDE_FROM=20 -DSW_IX2_WIDE_WAVES=4") 16 in the old
# 4-wave form without it and 20 in 4-wave workgroups; then C2 and its 1/8
# share.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r04ri20}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/intra_tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/intra_tests.log; exit 1; }
tail -1 $O/intra_tests.log
b() { tag=$1; shift; timeout -k 10 600 python3 bench.py --no-cpu-baseline "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag FAILED"; tail -20 $O/$tag.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/$tag.json').read().strip().split(chr(10))[-1]); r=d.get('reference_scoring',{})
print('$tag', d['value'], d['ms_per_step'], d['kernels'], r.get('value'), d.get('parity_sample_ok'), (d.get('sustained') or {}).get('value'))"; }
A4=ece1782-smith-waterman-cuda_amd/lib/ab4/libswamd.so
b c5_ri20_w12 --config c5
SW_INTRA_X2_RI=16 b c5_ri16_w12 --config c5
SW_INTRA_X2_RI=10 b c5_ri10_w4 --config c5
SW_AMD_LIB=$A4 SW_INTRA_X2_RI=16 b c5_ri16_w4_old --config c5
SW_AMD_LIB=$A4 b c5_ri20_w4 --config c5
b c5_ri20_w12b --config c5
SW_AMD_LIB=$A4 SW_INTRA_X2_RI=16 b c5_ri16_w4_oldb --config c5
b c2
b s8 --shard-of 8
echo RC=0
