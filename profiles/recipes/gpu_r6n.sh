# r06: signed-tx agreement sweep (smoke size first, then 20 batches of 1.25 M transactions)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6n
mkdir -p $O
cd $R
timeout -k 10 300 python -u tools/agree_signed_tx.py --batches 1 --txs 100000 --first 1000 --out $O/smoke.json || { echo "smoke sweep failed"; exit 1; }
timeout -k 10 1000 python -u tools/agree_signed_tx.py --batches ${NB:-20} --log $O/agree_batches.jsonl --out $O/agree_signed_tx.json
