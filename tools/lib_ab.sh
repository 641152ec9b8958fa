#!/bin/bash
# Build the kernels of git revision REV (default HEAD) into build/ab_<REV>/ so a
# workload can be timed against them beside the working tree's build, each in its
# own process on the same box (TCBEE_AB_LIB selects the library; tools only).
#   tools/lib_ab.sh build [REV]        (here, on the CPU)
#   tools/lib_ab.sh run REV -- CMD...  (on the GPU box: CMD with the old library)
set -eu
cd "$(dirname "$0")/.."
case "${1:-}" in
  build)
    rev=${2:-HEAD}
    d=build/ab_${rev//:/_}
    rm -rf "$d"; mkdir -p "$d/tcbee_amd/csrc" "$d/include"
    # REV "wt:NAME": the working tree as it is now, kept under build/ab_wt:NAME
    for f in tcbee_kernels.hip tcbee_capi.hip tcbee_pipe.hip tcbee_gen.h tcbee_internal.h tcbee_layout.h; do
      case $rev in wt:*) cp "tcbee_amd/csrc/$f" "$d/tcbee_amd/csrc/$f" ;;
                   *) git show "$rev:tcbee_amd/csrc/$f" > "$d/tcbee_amd/csrc/$f" ;; esac
    done
    case $rev in wt:*) cp include/tcbee_amd.h "$d/include/tcbee_amd.h" ;;
                 *) git show "$rev:include/tcbee_amd.h" > "$d/include/tcbee_amd.h" ;; esac
    # HIPEXTRA: extra compiler flags for this build (e.g. -DTCBEE_K1_LOAD_PRIO=3)
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function ${HIPEXTRA:-} -shared \
      -o "$d/libtcbee_amd.so" "$d/tcbee_amd/csrc/tcbee_kernels.hip" "$d/tcbee_amd/csrc/tcbee_capi.hip" "$d/tcbee_amd/csrc/tcbee_pipe.hip"
    echo "$d/libtcbee_amd.so" ;;
  run)
    rev=$2; shift 3
    TCBEE_AB_LIB=build/ab_${rev//:/_}/libtcbee_amd.so "$@" ;;
  *) echo "usage: $0 build [REV] | run REV -- CMD..." >&2; exit 2 ;;
esac
