#!/bin/bash
# r06d: the whole tree -- smoke, every GPU test, the default bench line, the CPU launch dry run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
bash tools/gpu_session.sh r06d smoke tests bench
