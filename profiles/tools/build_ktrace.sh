#!/bin/bash
# Diagnostic build: libdcue_hip.so with -DDCUE_KTRACE (per-workgroup phase timestamps, dcue_common.h)
# into scratch/ktrace/ (git-ignored); run profiles/tools/ktrace.py with DCUE_HIP_LIB pointing at it.
# (argument: the output directory, default scratch/ktrace; scratch/ is gpurun-ignored, so to run the
# trace on the GPU box build into a travelling, git-ignored directory such as ktrace_tmp/ and delete it
# afterwards.) Objects are kept in <dir>/obj and rebuilt only when their source is newer.
set -e
cd "$(dirname "$0")/../.."
OUTD=${1:-scratch/ktrace}
mkdir -p $OUTD/obj
ls amplifai-deepcontentrecommenders_amd/csrc/*.hip | xargs -P 8 -I{} sh -c 'f={}; b=$(basename $f .hip); o='$OUTD'/obj/$b.o; if [ -f $o ] && [ $o -nt $f ] && [ -z "$(find amplifai-deepcontentrecommenders_amd/csrc include -name "*.h" -newer $o)" ]; then exit 0; fi; extra=""; case $b in adam|optim) extra="-ffp-contract=off";; esac; /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I include -I amplifai-deepcontentrecommenders_amd/csrc -DDCUE_KTRACE $extra -c $f -o $o'
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -pthread -o $OUTD/libdcue_hip.so $OUTD/obj/*.o -L/opt/rocm/lib -lrccl
