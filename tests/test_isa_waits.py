"""Static race check on the compiled kernels (no GPU): every translation unit whose kernels read LDS by inline asm
(or pipeline LDS loads across MFMAs) is compiled for gfx950 to ISA, and tools/check_asm_waits.py verifies that no
instruction reads, copies or overwrites a register of an LDS load before the s_waitcnt lgkmcnt that retires it, or
of a vector-memory load before its s_waitcnt vmcnt (the saddr-form asm reloads of the W1 REV and W3i epilogues), or
overwrites the data registers of a 16-byte store within the two wait states the store still reads them (the W3i
inline-asm stores must pad themselves; hipcc only pads its own).
hipcc does not count inline-asm loads, so a register copy it inserts ahead of a hand-placed wait reads stale data
on some waves and launches only (found this way in the W1 tile seam, the wgrad reload and the first split-W1 build).
"""
import os
import shutil
import subprocess
import sys
import tempfile
from concurrent.futures import ThreadPoolExecutor

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, 'siren_amd', 'csrc')
TUS = ['tu_w1.hip', 'tu_w0.hip', 'tu_w4.hip', 'tu_w3.hip', 'tu_wide.hip', 'tu_jet.hip', 'tu_wide_jet.hip',
       'tu_train.hip', 'tu_w1x.hip', 'tu_hess.hip', 'tu_w3i_tt.hip', 'tu_w3i_tf.hip', 'tu_w3i_ft.hip', 'tu_w3i_ff.hip']

sys.path.insert(0, os.path.join(ROOT, 'tools'))


@pytest.mark.skipif(shutil.which('hipcc') is None and not os.path.exists('/opt/rocm/bin/hipcc'),
                    reason='hipcc not available')
def test_no_read_of_inflight_lds_load_registers():
    import check_asm_waits as C
    hipcc = shutil.which('hipcc') or '/opt/rocm/bin/hipcc'
    tmp = tempfile.mkdtemp(prefix='siren_isa_')

    def compile_one(tu):
        out = os.path.join(tmp, tu.replace('.hip', '.s'))
        subprocess.check_call([hipcc, '--offload-arch=gfx950', '-O3', '-std=c++17', '-mllvm',
                               '-pragma-unroll-threshold=1000000', '--cuda-device-only', '-S', '-I',
                               os.path.join(ROOT, 'include'), '-o', out, os.path.join(CSRC, tu)],
                              stderr=subprocess.DEVNULL)
        return tu, out

    try:
        with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 2)) as ex:
            outs = list(ex.map(compile_one, TUS))
        bad = []
        for tu, path in outs:
            import re
            s = open(path).read()
            for nm in re.findall(r'\n(_Z\w+):', s):
                i = s.find('\n' + nm + ':')
                j = s.find('.Lfunc_end', i)
                body = s[i:j].split('\n')
                probs = C.check(body, nm) + C.check_vmem(body, nm) + C.check_store_data(body, nm)
                if probs:
                    bad.append('%s %s: %d (first: %s)' % (tu, nm, len(probs), probs[0][1]))
        assert not bad, '\n'.join(bad)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
