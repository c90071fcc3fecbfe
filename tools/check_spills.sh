# Fails when a hot kernel of epi.hip spills VGPRs (control flow added to a 256-VGPR loop can
# turn into hundreds of scratch spills and a several-fold slowdown without any other symptom).
cd "$(dirname "$0")/../gmat_amd/csrc" || exit 1
/opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -x hip -c epi.hip -o /tmp/_spill_check.o \
  -Rpass-analysis=kernel-resource-usage 2>&1 |
  awk '/Function Name:/ {name=$NF} /VGPRs Spill:/ {n=$(NF-1); if (n+0 > 0 && name ~ /(lr_screen|mx_screen|side_gemm|screen_kernel)/) {print "SPILL", n, name; bad=1}} END {exit bad}'
