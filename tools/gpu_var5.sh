set -o pipefail
mkdir -p gpurun_out/var
for P in image_w2 hypernet sdf; do
  timeout -k 10 120 python tools/profile_paths.py $P > gpurun_out/var/b_$P.json 2>/dev/null && echo "base $P $(cut -c1-100 gpurun_out/var/b_$P.json)" || exit 1
  for L in tools/probe/lib_mm6.so tools/probe/lib_mm7.so; do
    SIREN_AMD_LIB=$L timeout -k 10 120 python tools/profile_paths.py $P > gpurun_out/var/x_$P.json 2>/dev/null && echo "$(basename $L) $P $(cut -c1-100 gpurun_out/var/x_$P.json)" || exit 1
  done
  timeout -k 10 120 python tools/profile_paths.py $P > gpurun_out/var/b_$P.json 2>/dev/null && echo "base $P $(cut -c1-100 gpurun_out/var/b_$P.json)" || exit 1
done
