set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python scripts/kmeans_variants.py --k 9984 --variants 14,17,18 --acc none --rounds 3 --out gpurun_out/variants_pipe4.json > gpurun_out/variants_pipe4.log 2>&1
