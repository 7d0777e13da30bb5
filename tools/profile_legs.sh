#!/bin/bash
# rocprofv3 evidence for bench.py's side measurements, one leg at a time (bench.py --only LEG), so
# each trace holds exactly that leg's launches:
#   OUT/LEG/prof       --kernel-trace --stats        (per-kernel durations; tools/kernel_grid_stats.py)
#   OUT/LEG/pmc_fetch  --pmc FETCH_SIZE              (own pass, --kernel-trace only)
#   OUT/LEG/pmc_write  --pmc WRITE_SIZE              (own pass)
#   OUT/LEG/leg.json   the leg's JSON line from the kernel-trace run
# Every step under its own time limit; anything but exit 0 ends the script (no further GPU steps).
#   usage: tools/profile_legs.sh TAG [legs...]     legs: spmm16 spmv_shapes cg_single cg_multi
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
TAG=${1:-legs}
shift
LEGS=${*:-spmm16 spmv_shapes cg_single cg_multi}
export TMPDIR=/tmp
for leg in $LEGS; do
    OUT=$PWD/gpurun_out/$TAG/$leg
    mkdir -p "$OUT"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o leg \
        -- python3 bench.py --only "$leg" --no-cpu >"$OUT/leg.json" 2>"$OUT/prof.err"
    rc=$?; echo "$leg prof rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/prof.err"; exit $rc; }
    for c in FETCH_SIZE WRITE_SIZE; do
        d=pmc_$(echo $c | cut -d_ -f1 | tr A-Z a-z)
        timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$OUT/$d" -o leg \
            -- python3 bench.py --only "$leg" --no-cpu >"$OUT/$d.json" 2>"$OUT/$d.err"
        rc=$?; echo "$leg $c rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/$d.err"; exit $rc; }
    done
done
echo "profile_legs $TAG done"
