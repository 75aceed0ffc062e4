# final ECDSA library: GPU suite, smoke, PMC C3/C5, evidence lines C3/C5/c3h (+ rocprof)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu_r3r.sh || exit 1
WLS="c3 c5 c3h c2" PROF="c3 c5" bash tools/gpu_evidence_r3.sh || exit 1
