set -e
mkdir -p gpurun_out/pf2
for s in "1000 44426" "400 44426" "2000 44426" "1000 177704" "300 70001"; do
  set -- $s
  timeout -k 5 60 tools/probe_pf $1 $2 5 > gpurun_out/pf2/n$1_p$2.txt 2> gpurun_out/pf2/n$1_p$2.err
done
echo done
