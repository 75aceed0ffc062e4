# P-256/secp256k1 formula glue A/B (ab_libs/ec_base, ec_z3, ec_sub) on C3, then
# the SQ_INSTS_VALU pass of the in-tree library (ec_sub) on a 2^22 C3 step
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
TAGS="ec_base ec_z3 ec_sub" TEST=tests/test_gpu_ecdsa.py WL=c3 STEPS=3 bash tools/gpu_ab.sh || exit 1
TAGS="ec_sub ec_base" TEST=tests/test_fp29_asm.py WL=c3 STEPS=3 bash tools/gpu_ab.sh || exit 1
O=$R/gpurun_out/pmc_c3sub
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d /tmp/pmc_1 -o p -- python3 $R/bench.py --workload c3 --batch-log2 22 --steps 1 --warmup 0 --no-cpu-baseline > $O/pass1.log 2>&1 || { echo "pmc failed"; tail -5 $O/pass1.log; exit 1; }
find /tmp/pmc_1 -name "*counter_collection.csv" -exec cp {} $O/pass1.csv \;
ls -la $O
