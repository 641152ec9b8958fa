#!/bin/bash
# Build the kernels of git revision REV (default HEAD) into ab/ab_<REV>/ so a
# workload can be timed against them beside the working tree's build, each in its
# own process on the same box (TCBEE_AB_LIB selects the library; tools only).
#   tools/lib_ab.sh build [REV]        (here, on the CPU)
#   tools/lib_ab.sh run REV -- CMD...  (on the GPU box: CMD with the old library)
# REV "wt:NAME": the working tree as it is now, kept under ab/ab_wt_NAME;
# HIPEXTRA: extra compiler flags for that build (build-time experiment knobs, -D...)
set -eu
cd "$(dirname "$0")/.."
case "${1:-}" in
  build)
    rev=${2:-HEAD}
    d=ab/ab_${rev//:/_}
    rm -rf "$d"; mkdir -p "$d/tcbee_amd/csrc" "$d/include"
    case $rev in
      wt:*) cp tcbee_amd/csrc/*.hip tcbee_amd/csrc/*.h "$d/tcbee_amd/csrc/"
            cp include/tcbee_amd.h "$d/include/tcbee_amd.h" ;;
      *) for f in $(git ls-tree --name-only "$rev" tcbee_amd/csrc/ | grep -E '\.(hip|h)$'); do
           git show "$rev:$f" > "$d/$f"
         done
         git show "$rev:include/tcbee_amd.h" > "$d/include/tcbee_amd.h" ;;
    esac
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function ${HIPEXTRA:-} -shared \
      -o "$d/libtcbee_amd.so" "$d"/tcbee_amd/csrc/*.hip
    echo "$d/libtcbee_amd.so" ;;
  run)
    rev=$2; shift 3
    TCBEE_AB_OPTIN=1 TCBEE_AB_LIB=ab/ab_${rev//:/_}/libtcbee_amd.so "$@" ;;
  *) echo "usage: $0 build [REV] | run REV -- CMD..." >&2; exit 2 ;;
esac
