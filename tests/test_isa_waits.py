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

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, 'siren_amd', 'csrc')
TUS = ['tu_w1.hip', 'tu_w1deep.hip', 'tu_w1nt.hip', 'tu_w0.hip', 'tu_w4.hip', 'tu_w3.hip', 'tu_wide.hip', 'tu_jet.hip', 'tu_wide_jet.hip',
       'tu_train.hip', 'tu_w1x.hip', 'tu_hess.hip', 'tu_w3i_tt.hip', 'tu_w3i_tf.hip', 'tu_w3i_ft.hip', 'tu_w3i_ff.hip',
       'tu_qfi.hip', 'tu_widei_fa.hip', 'tu_widei_ra.hip']

sys.path.insert(0, os.path.join(ROOT, 'tools'))


def _compile_and_check(tu):
    """(tu, problems) for one translation unit: hipcc to ISA, then the three checks on every kernel in it."""
    import re
    import check_asm_waits as C
    hipcc = shutil.which('hipcc') or '/opt/rocm/bin/hipcc'
    tmp = tempfile.mkdtemp(prefix='siren_isa_')
    try:
        out = os.path.join(tmp, tu.replace('.hip', '.s'))
        subprocess.check_call([hipcc, '--offload-arch=gfx950', '-O3', '-std=c++17', '-mllvm',
                               '-pragma-unroll-threshold=1000000', '--cuda-device-only', '-S', '-I',
                               os.path.join(ROOT, 'include'), '-o', out, os.path.join(CSRC, tu)],
                              stderr=subprocess.DEVNULL)
        s = open(out).read()
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    bad = []
    for nm in re.findall(r'\n(_Z\w+):', s):
        i = s.find('\n' + nm + ':')
        j = s.find('.Lfunc_end', i)
        body = s[i:j].split('\n')
        probs = (C.check(body, nm) + C.check_vmem(body, nm) + C.check_store_data(body, nm) + C.check_flat(body, nm) +
                 C.check_private(body, nm))
        if probs:
            bad.append('%s %s: %d (first: %s)' % (tu, nm, len(probs), probs[0][1]))
    return bad


@pytest.mark.skipif(shutil.which('hipcc') is None and not os.path.exists('/opt/rocm/bin/hipcc'),
                    reason='hipcc not available')
def test_no_read_of_inflight_lds_load_registers():
    from concurrent.futures import ProcessPoolExecutor
    with ProcessPoolExecutor(max_workers=min(8, os.cpu_count() or 2)) as ex:
        bad = [b for res in ex.map(_compile_and_check, TUS) for b in res]
    assert not bad, '\n'.join(bad)


def _walk_isa(text):
    import check_asm_waits as C
    body = ['_Zk:'] + [ln.strip() for ln in text.strip().split('\n')]
    return C.check(body, 'k') + C.check_vmem(body, 'k')


def test_checker_follows_fall_through_labels_and_back_edges():
    # a load in flight across a fall-through label is still checked after it
    assert _walk_isa("""
        ds_read_b128 v[0:3], v10
    .LBB0_1:
        v_add_f32 v4, v0, v1
        s_endpgm""")
    # ... and across a loop back-edge (issued at the bottom, read at the head before any wait)
    assert _walk_isa("""
    .LBB0_1:
        v_add_f32 v4, v0, v1
        global_load_dwordx4 v[0:3], v12, s[0:1]
        s_cbranch_scc1 .LBB0_1
        s_waitcnt vmcnt(0)
        s_endpgm""")
    # a wait on every path retires it
    assert not _walk_isa("""
        ds_read_b128 v[0:3], v10
        s_cbranch_scc1 .LBB0_2
        s_waitcnt lgkmcnt(0)
        s_branch .LBB0_3
    .LBB0_2:
        s_waitcnt lgkmcnt(0)
    .LBB0_3:
        v_add_f32 v4, v0, v1
        s_endpgm""")
    # a path that skips the wait is reported
    assert _walk_isa("""
        ds_read_b128 v[0:3], v10
        s_cbranch_scc1 .LBB0_3
        s_waitcnt lgkmcnt(0)
    .LBB0_3:
        v_add_f32 v4, v0, v1
        s_endpgm""")


def test_checker_correlates_flag_branches():
    # hipcc's lowering of `if (c) wait(0) else wait(4)`: the flag pair set on one path makes the second branch's
    # direction known, so the path that would skip both waits is infeasible and nothing is reported
    assert not _walk_isa("""
        global_load_dwordx4 v[0:3], v12, s[4:5]
        s_mov_b64 s[0:1], -1
        s_and_b64 vcc, exec, s[12:13]
        s_cbranch_vccz .LBB0_2
        s_waitcnt vmcnt(0)
        s_mov_b64 s[0:1], 0
    .LBB0_2:
        s_andn2_b64 vcc, exec, s[0:1]
        s_cbranch_vccnz .LBB0_4
        s_waitcnt vmcnt(0)
    .LBB0_4:
        v_add_f32 v4, v0, v1
        s_endpgm""")
    # the same shape with the second wait missing is reported
    assert _walk_isa("""
        global_load_dwordx4 v[0:3], v12, s[4:5]
        s_mov_b64 s[0:1], -1
        s_and_b64 vcc, exec, s[12:13]
        s_cbranch_vccz .LBB0_2
        s_waitcnt vmcnt(0)
        s_mov_b64 s[0:1], 0
    .LBB0_2:
        s_andn2_b64 vcc, exec, s[0:1]
        s_cbranch_vccnz .LBB0_4
    .LBB0_4:
        v_add_f32 v4, v0, v1
        s_endpgm""")


@pytest.mark.skipif(shutil.which('hipcc') is None and not os.path.exists('/opt/rocm/bin/hipcc'),
                    reason='hipcc not available')
def test_split_reverse_tile_loop_has_no_compiler_vmcnt():
    """The split-bf16 reverse (X_REV) counts every vector-memory operation of its tile loop itself: the next tile's
    cos blocks and inputs are inline-asm loads waited by the tile start's counted wait (w1x_kernel.hpp x_next_cos /
    x_next_issue). A compiler load in the loop brings back a compiler s_waitcnt vmcnt, which does not know the asm
    operations and drains the weight ring (the round-5 tile-start drain). Only asm waits may appear after the tile
    loop's header."""
    import re
    hipcc = shutil.which('hipcc') or '/opt/rocm/bin/hipcc'
    tmp = tempfile.mkdtemp(prefix='siren_isa_')
    try:
        out = os.path.join(tmp, 'tu_w1x.s')
        subprocess.check_call([hipcc, '--offload-arch=gfx950', '-O3', '-std=c++17', '-mllvm',
                               '-pragma-unroll-threshold=1000000', '--cuda-device-only', '-S', '-I',
                               os.path.join(ROOT, 'include'), '-o', out, os.path.join(CSRC, 'tu_w1x.hip')],
                              stderr=subprocess.DEVNULL)
        s = open(out).read()
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    names = re.findall(r'\n(_ZN5siren10w1x_kernelILi3ELi[23]ELi4E\w+):', s)
    assert len(names) == 2, names
    for nm in names:
        i = s.find('\n' + nm + ':')
        body = [ln.strip() for ln in s[i:s.find('.Lfunc_end', i)].split('\n')]
        headers = [k for k, ln in enumerate(body) if 'Loop Header' in ln]
        assert headers, nm
        in_asm, waits = False, []
        for k, ln in enumerate(body):
            if ln.startswith(';;#ASMSTART'):
                in_asm = True
            elif ln.startswith(';;#ASMEND'):
                in_asm = False
            elif not in_asm and ln.startswith('s_waitcnt') and 'vmcnt' in ln and k > headers[-1]:
                waits.append(ln)
        assert not waits, '%s: compiler vmcnt waits in the tile loop: %s' % (nm, waits)
