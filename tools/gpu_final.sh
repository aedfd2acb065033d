set -o pipefail
SQ_PASSES=1 bash tools/profile_round.sh r03y || exit 1
for P in w3_theta sdf; do
  timeout -k 10 120 python tools/profile_paths.py $P > gpurun_out/var/base2_$P.json 2>/dev/null && echo "base $P $(cat gpurun_out/var/base2_$P.json | cut -c1-120)"
  for L in tools/probe/lib_w3ip6.so tools/probe/lib_w3ip7.so; do
    SIREN_AMD_LIB=$L timeout -k 10 120 python tools/profile_paths.py $P > gpurun_out/var/x_$P.json 2>/dev/null && echo "$(basename $L) $P $(cat gpurun_out/var/x_$P.json | cut -c1-120)"
  done
done
