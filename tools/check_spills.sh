# Fails when a hot scan kernel (epi_*.hip) spills more than a few VGPRs (control flow added to a
# 256-VGPR loop can turn into hundreds of scratch spills and a several-fold slowdown without any
# other symptom; a handful of spills outside the loops, as lr_screen_kernel<2> has, are harmless).
# The phase-stamped prefilter build (GMAT_PF_STAMPS, diagnostics only) is reported but not checked.
cd "$(dirname "$0")/../gmat_amd/csrc" || exit 1
for f in epi_prefilter.hip epi_screen.hip epi_refine.hip; do
  /opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -fno-slp-vectorize -x hip -c $f -o /tmp/_spill_check.o \
    -Rpass-analysis=kernel-resource-usage 2>&1
done |
  awk '/Function Name:/ {name=$(NF-1); if (name ~ /prefilter_pass_kernelILb1ELb1ELb1E/) name = "stamped:" name} /VGPRs Spill:/ {n=$(NF-1); if (n+0 > 8 && name !~ /^stamped/ && name ~ /(lr_screen|mx_screen|side_gemm|screen_kernel|prefilter_pass)/) {print "SPILL", n, name; bad=1} else if (n+0 > 0 && name ~ /(lr_screen|mx_screen|side_gemm|screen_kernel|prefilter_pass)/) print "spill (ok)", n, name} END {exit bad}'
