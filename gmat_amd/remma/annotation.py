"""Hit annotation -- drop-in for gmat.remma.annotation.annotation_snp_pos (annotation.py:22-73)."""
from .. import dist


@dist.on_root
def annotation_snp_pos(res_file, bed_file, p_cut=1, dis=0, ld_file=None, r2=0.2):
    """Rewrite res_file's header with .bim columns and keep rows with p <= p_cut whose SNPs
    are on different chromosomes or more than `dis` bp apart; writes res_file + '.anno'
    (and '.anno.ld' without the pairs in LD above r2 when ld_file is given)."""
    info = []
    with open(bed_file + ".bim") as f:
        for line in f:
            info.append(" ".join(line.split()))
    with open(res_file) as fin, open(res_file + ".anno", "w") as fout:
        hdr = fin.readline().split()
        fout.write(" ".join([hdr[0], "snp0_chr", "snp0_ID", "snp0_cm", "snp0_bp", "snp0_allele1", "snp0_allele2",
                             hdr[1], "snp1_chr", "snp1_ID", "snp1_cm", "snp1_bp", "snp1_allele1", "snp1_allele2"]))
        fout.write(" " + " ".join(hdr[2:]) + "\n")
        for line in fin:
            a = line.split()
            s0 = info[int(a[0])].split()
            s1 = info[int(a[1])].split()
            if float(a[-1]) <= p_cut and (s0[0] != s1[0] or abs(float(s0[3]) - float(s1[3])) > dis):
                fout.write(" ".join([a[0], info[int(a[0])], a[1], info[int(a[1])]]) + " " + " ".join(a[2:]) + "\n")
    if ld_file is not None:
        ld = set()
        with open(ld_file) as f:
            f.readline()
            for line in f:
                a = line.split()
                if float(a[-1]) > r2:
                    ld.add(a[2] + " " + a[5])
                    ld.add(a[5] + " " + a[2])
        with open(res_file + ".anno") as fin, open(res_file + ".anno.ld", "w") as fout:
            fout.write(fin.readline())
            for line in fin:
                a = line.split()
                if a[2] + " " + a[9] not in ld:
                    fout.write(line)
    return 0
