set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python tools/env_ab.py --variants ";LEOEC_GFBIT_WG=128;LEOEC_GFBIT_WG=512;LEOEC_GFBIT_WG=1024;LEOEC_GFBIT_WG=5121;LEOEC_GFBIT_WG=10241;LEOEC_GFBIT_CEIL=1" > gpurun_out/ab_cauchy3.log 2>&1
