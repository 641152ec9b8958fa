# Config 2 under the variants library, K1 with TCBEE_NT=0 / 1 (non-temporal index
# loads and record / side-word stores), alternating processes (tools/c2_warm.py).
set -u
V=tcbee_amd/lib/libtcbee_amd_variants.so
for r in 1 2; do
  for nt in 0 1; do
    echo "=== NT=$nt round $r"
    TCBEE_NT=$nt TCBEE_AB_LIB=$V timeout -k 10 120 python tools/c2_warm.py --rounds 1 --idle 0.5 --legs 1000:1000 2>/dev/null | tail -1 || exit $?
  done
done
