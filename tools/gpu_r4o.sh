set -o pipefail
bash tools/gpu_tests.sh r4o || exit 1
bash tools/measure_round.sh r04 && echo measured
