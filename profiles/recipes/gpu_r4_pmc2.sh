# Round-4 PMC re-take of C4 and C5 on the round-4 library (one counter group per
# pass, tools/gpu_pmc.sh), for traffic = HBM with the ladder's MALL split
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
TAG=r4_c4 WL=c4 C4TXS=262144 bash tools/gpu_pmc.sh > gpurun_out/pmc_r4_c4.txt 2>&1 || { echo "c4 pmc failed"; tail -5 gpurun_out/pmc_r4_c4.txt; exit 1; }
TAG=r4_c5 WL=c5 LOG2=22 bash tools/gpu_pmc.sh > gpurun_out/pmc_r4_c5.txt 2>&1 || { echo "c5 pmc failed"; tail -5 gpurun_out/pmc_r4_c5.txt; exit 1; }
grep -h '"metric"' gpurun_out/pmc_r4_c4/pass1.log gpurun_out/pmc_r4_c5/pass1.log | cut -c1-200
echo done
