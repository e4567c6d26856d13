set -o pipefail
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r04_blasname -o run --output-format csv -- python3 $R/tools/blas_kernel_name.py 10000 16384 > $R/gpurun_out/r04_blasname.log 2>&1
