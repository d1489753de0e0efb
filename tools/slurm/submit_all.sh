#!/usr/bin/env bash
# Submit the GPU-count sweep as SLURM jobs (the role of the reference's mpi/submit_all.sh, which
# submitted 32/128/512-node BlueGene/L jobs). One job per GPU count on one MI355X node; each job
# runs tools/slurm/mi355x_sweep.sbatch, which launches one rank per GPU with srun.
#
#   tools/slurm/submit_all.sh [GPU_COUNTS...]        default: 1 2 4 8
#   env: PARTITION=<name>  TIME=00:10:00  MODE=vector|scalar  DRY_RUN=1 (print, do not submit)
#        EXTRA="--dtypes=INT,DOUBLE --retries=5"  (passed to reduce_xgmi)
set -euo pipefail
HERE="$(cd "$(dirname "$0")" && pwd)"
COUNTS=("$@")
[ ${#COUNTS[@]} -eq 0 ] && COUNTS=(1 2 4 8)
export MODE="${MODE:-vector}" EXTRA="${EXTRA:-}"  # reach the job through --export ALL
PART_ARG=()
[ -n "${PARTITION:-}" ] && PART_ARG=(-p "$PARTITION")
for G in "${COUNTS[@]}"; do
  case "$G" in 1|2|3|4|5|6|7|8) ;; *) echo "GPU count must be 1..8 (one node), got $G" >&2; exit 2 ;; esac
  cmd=(sbatch "${PART_ARG[@]}" --nodes 1 --ntasks-per-node "$G" --gpus-per-node "$G" -t "${TIME:-00:10:00}"
       -o "./jobstdout-%j" --export ALL "$HERE/mi355x_sweep.sbatch")
  if [ -n "${DRY_RUN:-}" ]; then echo "${cmd[*]}"; else "${cmd[@]}"; fi
done
