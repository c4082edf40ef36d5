set -o pipefail
bash tools/gpu_job.sh rocprof r6a CNNModel TransformerModel RNNModel || exit 1
