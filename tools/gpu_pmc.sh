set -e -o pipefail
bash tools/pmc_micro.sh f44 4 4 512 512 128 3 1 1 1 fwd bf16 3
bash tools/pmc_micro.sh f99 9 9 128 128 32 3 1 1 1 fwd bf16 3
