# rank 0's part of the 8-way split (tools/split_part.py, 8 scans) under several environment settings,
# alternating, twice: bash tools/part_env_ab.sh OUT 'name=ENV=val,ENV2=val' 'name2=' ...
out=gpurun_out/$1; shift
mkdir -p $out
for rep in 1 2; do
  for arm in "$@"; do
    name=${arm%%=*}; envs=${arm#*=}
    env_args=$(echo "$envs" | tr ',' ' ')
    env $env_args timeout -k 10 200 python3 tools/split_part.py 0 ${WAYS:-8} 8 > $out/$name.$rep.log 2>&1 || { echo "arm $name failed"; tail -5 $out/$name.$rep.log; exit 1; }
    python3 -c "
import re, statistics
t = [float(m.group(1)) for m in re.finditer(r'rows, ([0-9.]+) ms', open('$out/$name.$rep.log').read())]
print('%-10s rep $rep: median %.3f ms, min %.3f (%d scans)' % ('$name', statistics.median(t), min(t), len(t)))"
  done
done
