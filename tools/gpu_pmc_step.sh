# r06 PMC campaign: every bench line's own counters on the r06 library. Per workload,
# three counter passes (SQ group, FETCH_SIZE, WRITE_SIZE) over --steps 1 and over
# --steps 2 (--warmup 0): tools/pmc_step.py takes the difference = one timed step.
# WL: "tag|bench args|algorithmic bytes per unit" entries separated by ';'
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc6
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
SQ="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
IFS=';' read -ra ENTRIES <<< "$WL"
for e in "${ENTRIES[@]}"; do
  IFS='|' read -r tag args alg <<< "$e"
  D=$O/$tag
  mkdir -p $D
  for st in 1 2; do
    for g in A B C; do
      case $g in A) grp="$SQ";; B) grp="FETCH_SIZE";; C) grp="WRITE_SIZE";; esac
      rm -rf /tmp/pmc_x
      timeout -s KILL 170 rocprofv3 --pmc $grp --output-format csv -d /tmp/pmc_x -o p -- python3 $R/bench.py $args --steps $st --warmup 0 --no-clock --no-cpu-baseline > $D/s${st}_$g.log 2>&1 || { echo "pmc $tag s$st $g failed"; tail -5 $D/s${st}_$g.log; exit 1; }
      find /tmp/pmc_x -name "*counter_collection.csv" -exec cp {} $D/s${st}_$g.csv \;
      [ $g = A ] && [ $st = 2 ] && { grep -h '^{' $D/s2_A.log | tail -1 > $D/s2_line.json; }
      echo "$tag s$st $g done"
    done
  done
  python3 $R/tools/pmc_step.py $D $tag "$args" $alg > $O/r06_pmc_$tag.json && python3 -c "
import json; d = json.load(open('$O/r06_pmc_$tag.json')); t = d['total']['derived']
print('$tag', 'units', round(d['units_per_step']), 'fabric B/unit', round(d['l2_fabric_bytes_per_unit']), 'hbm B/unit', round(d['hbm_bytes_per_unit']), 'valu_busy', round(t.get('valu_busy_est_4cyc', 0), 3), 'valu/lane', round(t.get('valu_lane_insts_per_lane', 0)))" || exit 1
done
