set -o pipefail
mkdir -p gpurun_out/w3i
timeout -k 10 400 python -u -m pytest tests/test_gpu_w3i.py -x -v --timeout 200 --timeout-method thread > gpurun_out/w3i/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/w3i/tests.log; exit 1; }
tail -3 gpurun_out/w3i/tests.log
for p in w3_theta sdf; do for f in 0 4; do
  SIREN_FLAGS=$f timeout -k 10 120 python tools/profile_paths.py $p > gpurun_out/w3i/t_${p}_$f.json 2>gpurun_out/w3i/t_${p}_$f.err || { echo "timing $p $f failed"; tail -5 gpurun_out/w3i/t_${p}_$f.err; exit 1; }
  echo "$p flags=$f: $(cat gpurun_out/w3i/t_${p}_$f.json)"
done; done
