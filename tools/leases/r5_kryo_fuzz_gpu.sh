set -o pipefail
O=gpurun_out/r5kfuzz; mkdir -p $O
timeout -k 10 600 python -u tools/agree_kryo_fuzz.py --rounds 100000 --calls 8 --out $O/r05_agreement_kryo_fuzz.json > $O/run.log 2>&1 || { tail -30 $O/run.log; exit 1; }
tail -2 $O/run.log
