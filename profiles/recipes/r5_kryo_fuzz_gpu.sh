set -o pipefail
O=gpurun_out/r5kfuzz; mkdir -p $O
CORDAHIP_TRACE=1 timeout -k 10 600 python -u tools/agree_kryo_fuzz.py --rounds ${ROUNDS:-100000} --calls ${CALLS:-8} --txcomp-rounds ${TXR:-100000} --out $O/r05_agreement_kryo_fuzz.json > $O/run.log 2> $O/trace.log || { tail -30 $O/run.log $O/trace.log; exit 1; }
tail -2 $O/run.log | cut -c1-800
grep -E "^\[agree\]|component call" $O/trace.log > $O/passes.log || true
cat $O/passes.log
