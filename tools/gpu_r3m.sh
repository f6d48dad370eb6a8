set -o pipefail
export TMPDIR=/tmp
timeout -k 10 1100 bash tools/evidence_r03.sh gpurun_out/r3m c7da401 > gpurun_out/r3m.log 2>&1; echo "rc=$?" >> gpurun_out/r3m.log
