# Wide intra image (v_pk_fma_f16 with op_sel instead of v_perm_b32 + add):
# intra parity with each wide shape forced, then C5 A/B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/wide
mkdir -p $O
T="python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k intra --timeout 120 --timeout-method thread"
SW_INTRA_X2_WIDE=8 SW_INTRA_X2_RI=16 timeout -k 10 300 $T > $O/p16_8.log 2>&1 && \
SW_INTRA_X2_WIDE=12 SW_INTRA_X2_RI=16 timeout -k 10 300 $T > $O/p16_12.log 2>&1 && \
SW_INTRA_X2_WIDE=4 SW_INTRA_X2_RI=12 timeout -k 10 300 $T > $O/p12_4.log 2>&1 && \
SW_INTRA_X2_WIDE=8 SW_INTRA_X2_RI=8 timeout -k 10 300 $T > $O/p8_8.log 2>&1 && \
B="python3 bench.py --config c5 --no-cpu-baseline" && \
timeout -k 10 300 $B > $O/base.json 2> $O/base.err && \
SW_INTRA_X2_WIDE=8 timeout -k 10 300 $B > $O/w16_8.json 2> $O/w16_8.err && \
SW_INTRA_X2_WIDE=12 timeout -k 10 300 $B > $O/w16_12.json 2> $O/w16_12.err && \
SW_INTRA_X2_RI=12 timeout -k 10 300 $B > $O/b12.json 2> $O/b12.err && \
SW_INTRA_X2_WIDE=4 SW_INTRA_X2_RI=12 timeout -k 10 300 $B > $O/w12_4.json 2> $O/w12_4.err && \
SW_INTRA_X2_WIDE=8 SW_INTRA_X2_RI=12 timeout -k 10 300 $B > $O/w12_8.json 2> $O/w12_8.err
rc=$?; echo RC=$rc; for f in p16_8 p16_12 p12_4 p8_8; do tail -1 $O/$f.log; done
for f in base w16_8 w16_12 b12 w12_4 w12_8; do [ -f $O/$f.json ] && python3 -c "
import json
d=json.loads(open('$O/$f.json').read().strip().split(chr(10))[-1]); r=d.get('reference_scoring',{})
print('$f', d['value'], d['kernels']['intra'], d['kernel_ms_per_scan']['sw_intra'], r.get('value'), r.get('kernel_ms_per_scan',{}).get('sw_intra'))"; done; exit $rc
