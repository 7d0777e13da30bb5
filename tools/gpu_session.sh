#!/bin/bash
# One GPU-box session: smoke -> GPU parity tests -> bench -> rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; a crash / abort / timeout (anything but exit 0 or a
# plain test failure, exit 1) ends the session so nothing else touches a possibly-faulted GPU.
#   usage: tools/gpu_session.sh TAG [steps...]
#   steps: smoke tests bench prof pmc readceil
#          legs:LEG[,LEG]            tools/profile_legs.sh (kernel trace + FETCH/WRITE passes per bench leg)
#          counters:LEG:REGEX        tools/pmc_passes.sh on `bench.py --only LEG` for kernels matching REGEX
#          pytest:PATH                one test file / node id, -m gpu
#          py:SCRIPT[:ARGS]          a lab script (python3 SCRIPT ARGS, 300 s limit)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
TAG=${1:-run}
shift
STEPS=${*:-smoke tests bench prof}
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp

stop_unless_ok() {  # $1 rc, $2 step
    if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then
        echo "STOP: $2 exited $1 (fault/abort/timeout) -- no further GPU steps"
        exit "$1"
    fi
}

for s in $STEPS; do
    case $s in
    smoke)
        timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" >"$OUT/smoke.log" 2>&1
        rc=$?; echo "smoke rc=$rc"; tail -3 "$OUT/smoke.log"; stop_unless_ok $rc smoke ;;
    tests)
        timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -rf >"$OUT/pytest_gpu.log" 2>&1
        rc=$?; echo "pytest rc=$rc"; tail -25 "$OUT/pytest_gpu.log"; stop_unless_ok $rc tests ;;
    bench)
        timeout -k 10 600 python bench.py >"$OUT/bench.json" 2>"$OUT/bench.err"
        rc=$?; echo "bench rc=$rc"; cat "$OUT/bench.json"; tail -5 "$OUT/bench.err"; stop_unless_ok $rc bench ;;
    prof)
        timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o bench \
            -- python3 bench.py --no-cpu --no-cg --no-extras >"$OUT/prof_bench.json" 2>"$OUT/prof.err"
        rc=$?; echo "prof rc=$rc"; find "$OUT/prof" -name "*kernel_stats.csv" | head -3
        stop_unless_ok $rc prof ;;
    pmc)
        timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_fetch" -o bench \
            -- python3 bench.py --no-cpu --no-cg --no-extras >"$OUT/pmc_fetch.json" 2>"$OUT/pmc_fetch.err"
        rc=$?; echo "pmc fetch rc=$rc"; stop_unless_ok $rc pmc_fetch
        timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_write" -o bench \
            -- python3 bench.py --no-cpu --no-cg --no-extras >"$OUT/pmc_write.json" 2>"$OUT/pmc_write.err"
        rc=$?; echo "pmc write rc=$rc"; stop_unless_ok $rc pmc_write ;;
    pytest:*)
        timeout -k 10 900 python -m pytest ${s#pytest:} -m gpu -q -p no:cacheprovider -rf >"$OUT/pytest_sel.log" 2>&1
        rc=$?; echo "pytest ${s#pytest:} rc=$rc"; tail -15 "$OUT/pytest_sel.log"; stop_unless_ok $rc pytest ;;
    readceil)
        [ -x tools/read_ceiling ] || /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o tools/read_ceiling tools/read_ceiling.hip
        timeout -k 10 300 tools/read_ceiling >"$OUT/read_ceiling.txt" 2>&1
        rc=$?; echo "readceil rc=$rc"; cat "$OUT/read_ceiling.txt"; stop_unless_ok $rc readceil ;;
    legs:*)
        timeout -k 10 900 bash tools/profile_legs.sh "$TAG" $(echo "${s#legs:}" | tr , ' ')
        rc=$?; echo "legs rc=$rc"; stop_unless_ok $rc legs ;;
    counters:*)
        spec=${s#counters:}; leg=${spec%%:*}; re=${spec#*:}
        timeout -k 10 1200 bash tools/pmc_passes.sh "$OUT/counters_$leg" "$re" -- python3 bench.py --only "$leg" --no-cpu
        rc=$?; echo "counters $leg rc=$rc"; stop_unless_ok $rc counters ;;
    py:*)
        spec=${s#py:}; script=${spec%%:*}; args=""; [ "$spec" != "$script" ] && args=$(echo "${spec#*:}" | tr , ' ')
        timeout -k 10 300 python3 -u "$script" $args >"$OUT/$(basename "$script" .py).txt" 2>&1
        rc=$?; echo "py $script rc=$rc"; tail -40 "$OUT/$(basename "$script" .py).txt"; stop_unless_ok $rc py ;;
    *)
        echo "unknown step $s"; exit 2 ;;
    esac
done
echo "session $TAG done"
