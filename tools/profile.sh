#!/usr/bin/env bash
# rocprofv3 wrapper: one kernel-trace/stats run and one separate counter run
# (never combine --pmc with trace domains). Output under gpurun_out/<tag>_{trace,pmc}/.
#   usage: tools/profile.sh <tag> -- <program> [args...]
#   env:   PMC="FETCH_SIZE SQ_WAVES GRBM_GUI_ACTIVE" (default)
set -euo pipefail
TAG="$1"; shift
[ "$1" = "--" ] && shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
PMC="${PMC:-FETCH_SIZE SQ_WAVES GRBM_GUI_ACTIVE}"
mkdir -p gpurun_out
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "gpurun_out/${TAG}_trace" -o run --output-format csv -- "$@"
# shellcheck disable=SC2086
timeout -k 10 600 rocprofv3 --pmc $PMC -d "gpurun_out/${TAG}_pmc" -o run --output-format csv -- "$@"
python3 "$(dirname "$0")/prof_summary.py" "gpurun_out/${TAG}_trace" "gpurun_out/${TAG}_pmc"
