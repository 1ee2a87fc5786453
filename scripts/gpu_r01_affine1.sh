# Affine BLOSUM62 (BLAST 11/1 = open 12, extend 1 here) shape sweep on C2.
set -o pipefail
mkdir -p gpurun_out
SW_TUNE_SCORING=1:12:1 timeout -k 10 600 python3 scripts/tune_inter.py ${1:-32x8,32x16,48x8,64x8,16x16} ${2:-3072,2048,1536,1024} > gpurun_out/aff1.jsonl 2> gpurun_out/aff1.err
rc=$?; echo RC=$rc; cat gpurun_out/aff1.jsonl; tail -3 gpurun_out/aff1.err; exit $rc
