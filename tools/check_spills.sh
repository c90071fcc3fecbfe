# Fails when a hot kernel of epi.hip spills more than a few VGPRs (control flow added to a
# 256-VGPR loop can turn into hundreds of scratch spills and a several-fold slowdown without any
# other symptom; a handful of spills outside the loops, as lr_screen_kernel<2> has, are harmless).
cd "$(dirname "$0")/../gmat_amd/csrc" || exit 1
/opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -fno-slp-vectorize -x hip -c epi.hip -o /tmp/_spill_check.o \
  -Rpass-analysis=kernel-resource-usage 2>&1 |
  awk '/Function Name:/ {name=$(NF-1)} /VGPRs Spill:/ {n=$(NF-1); if (n+0 > 8 && name ~ /(lr_screen|mx_screen|side_gemm|screen_kernel|prefilter_pass)/) {print "SPILL", n, name; bad=1} else if (n+0 > 0 && name ~ /(lr_screen|mx_screen|side_gemm|screen_kernel|prefilter_pass)/) print "spill (ok)", n, name} END {exit bad}'
