set -o pipefail
OUT=r04h TAG=r04 bash tools/session.sh tests bench_c4 prof_c4 pmc_c4
