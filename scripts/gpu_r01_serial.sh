# C2: intra kernel concurrent (default) vs serial before the inter kernel
# (SW_INTRA_SERIAL=1: the inter kernel's time alone), long thresholds.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/serial
mkdir -p $O
B="python3 bench.py --no-cpu-baseline"
timeout -k 10 300 $B > $O/conc.json 2> $O/conc.err && \
SW_INTRA_SERIAL=1 timeout -k 10 300 $B > $O/serial.json 2> $O/serial.err && \
timeout -k 10 300 $B --long-threshold 3072 > $O/t3072.json 2> $O/t3072.err && \
timeout -k 10 300 $B --long-threshold 1536 > $O/t1536.json 2> $O/t1536.err
rc=$?; echo RC=$rc; for f in conc serial t3072 t1536; do python3 -c "
import json
d=json.loads(open('$O/$f.json').read().strip().split(chr(10))[-1]); r=d['reference_scoring']
print('$f', d['value'], d['ms_per_step'], d['kernel_ms_per_scan'], d['config']['long_subjects'], r['value'], r['kernel_ms_per_scan'])"; done; exit $rc
