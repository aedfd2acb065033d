set -o pipefail
mkdir -p gpurun_out/var
run() {  # path lib-or-base
  local P=$1 L=$2 t=base
  if [ "$L" != base ]; then t=$(basename $L .so); fi
  if [ "$L" = base ]; then timeout -k 10 120 python tools/profile_paths.py $P > gpurun_out/var/${t}_$P.json 2>/dev/null || return 1
  else SIREN_AMD_LIB=$L timeout -k 10 120 python tools/profile_paths.py $P > gpurun_out/var/${t}_$P.json 2>/dev/null || return 1; fi
  echo "$t $P $(python -c "import json;d=json.load(open('gpurun_out/var/${t}_$P.json'));print(d['ms_per_step'], d['frac_fp32_peak'])")"
}
for P in w0 poisson; do run $P base && run $P tools/probe/lib_ma.so && run $P base || exit 1; done
for P in image_w2 hypernet sdf; do run $P base && run $P tools/probe/lib_mb.so && run $P tools/probe/lib_mc.so && run $P base || exit 1; done
