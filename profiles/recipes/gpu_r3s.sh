# ECDSA part of the north-star sweep on the final kernels: EC batches
# [FIRST, FIRST + EC), every lane checked by the C oracle on the box's host threads
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r3s}
mkdir -p $O
cd $R
timeout -k 10 ${SWEEP_S:-1000} python -u tools/agree_1e9.py --oracle-all --ed 0 --ec ${EC:-3} --first ${FIRST:-0} --threads 16 --log $O/agree_log.jsonl > $O/agree.out 2>&1; rc=$?
tail -n 3 $O/agree.out
exit $rc
