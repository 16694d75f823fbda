# First GPU call of a session: GPU tests, smoke, headline bench (+ same-process eager baseline), kernel profile.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash bench/gpu_check.sh && bash bench/gpu_prof.sh gpurun_out/prof_start
