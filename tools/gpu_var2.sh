set -o pipefail
mkdir -p gpurun_out/var
for P in w1 w3_theta sdf; do
  SIREN_FLAGS=0 timeout -k 10 120 python tools/profile_paths.py $P > gpurun_out/var/base_$P.json 2>/dev/null || exit 1
  echo "base $P $(cat gpurun_out/var/base_$P.json)"
  for lib in tools/probe/lib_*.so; do
    t=$(basename $lib .so)
    case "$P:$t" in w1:lib_w1*|w3_theta:lib_w3i*|sdf:lib_w3i*) ;; *) continue;; esac
    SIREN_AMD_LIB=$lib timeout -k 10 120 python tools/profile_paths.py $P > gpurun_out/var/${t}_$P.json 2>/dev/null || exit 1
    echo "$t $P $(cat gpurun_out/var/${t}_$P.json)"
  done
done
