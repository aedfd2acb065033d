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
TUS = ['tu_w1.hip', 'tu_w1deep.hip', 'tu_widei_fb.hip', 'tu_w1nt.hip', 'tu_w0.hip', 'tu_w4.hip', 'tu_w3.hip', 'tu_wide.hip', 'tu_jet.hip', 'tu_wide_jet.hip',
       'tu_train.hip', 'tu_w1x.hip', 'tu_hess.hip', 'tu_w3i_tt.hip', 'tu_w3i_tf.hip', 'tu_w3i_ft.hip', 'tu_w3i_ff.hip',
       'tu_qfi.hip', 'tu_widei_fa.hip', 'tu_widei_ra.hip']

sys.path.insert(0, os.path.join(ROOT, 'tools'))


# kernels whose tile loop must hold no compiler s_waitcnt vmcnt (they count every vector-memory op themselves): the
# recompute W2 store, the fp32 reverse at every depth (the image / hypernet W2 backward; gx-only REV of the deep and
# notile forms) and the split-bf16 reverse. (The headline W1 body is not among them: its spill-free form measured slower,
# DESIGN.md §3.1.) A compiler load or scratch reload in the loop brings one back, and it drains the weight ring.
LOOP_WAIT_FREE = {
    'tu_w1.hip': [r'_ZN5siren9w1_kernelILi[123]ELi5E\w+', r'_ZN5siren9w1_kernelILi[123]ELi1E\w+'],
    'tu_w1deep.hip': [r'_ZN5siren9w1_kernelILi[45]ELi5E\w+'],
    'tu_w1nt.hip': [r'_ZN5siren9w1_kernelILi[1-5]ELi37E\w+'],
    'tu_w1x.hip': [r'_ZN5siren10w1x_kernelILi3ELi[23]ELi4E\w+'],
}


# kernels whose 16-byte stores are all tiles / kept jets / spill slots read back by a later kernel (or a later phase):
# every global_store_dwordx4 must carry the nontemporal hint (without it they evict the weight image
# from L2; qfi 4.96 -> 4.39 ms, w3i 5.91 -> 5.51 ms with it)
NT_STORE_KERNELS = {
    'tu_qfi.hip': [r'_ZN5siren14qfi_rev_kernelILi\dE\w+'],
    'tu_w3i_tt.hip': [r'_ZN5siren10w3i_kernelILi\dELb1ELb1E\w+'],
    'tu_hess.hip': [r'_ZN5siren11hess_kernelILb1E\w+'],
    'tu_widei_fb.hip': [r'_ZN5siren12widei_kernel\w+'],
}


def tile_loop_vmcnt_waits(body):
    """Compiler (non-asm) s_waitcnt vmcnt in the blocks of a kernel's last depth-1 loop (the persistent tile loop):
    its header block and every block hipcc marks `in Loop: Header=` that header, the latch included."""
    import re
    heads = [re.match(r'(\.LBB\w+):', ln).group(1) for ln in body
             if 'Loop Header: Depth=1' in ln and re.match(r'\.LBB\w+:', ln)]
    if not heads:
        return None
    hdr = heads[-1]
    tag = 'Header=' + hdr[2:]  # .LBB5_24 -> 'Header=BB5_24'
    in_loop = in_asm = False
    waits = []
    for ln in body:
        m = re.match(r'(\.LBB\w+):', ln)
        if m:
            in_loop = m.group(1) == hdr or tag + ' ' in ln + ' '
        elif ln.startswith('; %bb.'):
            in_loop = tag + ' ' in ln + ' '
        if ln.startswith(';;#ASMSTART'):
            in_asm = True
        elif ln.startswith(';;#ASMEND'):
            in_asm = False
        elif in_loop and not in_asm and ln.startswith('s_waitcnt') and 'vmcnt' in ln:
            waits.append(ln)
    return waits


def _compile_and_check(tu):
    """(tu, problems, loop waits) for one translation unit: hipcc to ISA, then the ISA checks on every kernel in it,
    and the tile-loop vmcnt scan of its LOOP_WAIT_FREE kernels ({name: [waits]})."""
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
    bad, loops, plain = [], {}, {}
    for nm in re.findall(r'\n(_Z\w+):', s):
        i = s.find('\n' + nm + ':')
        j = s.find('.Lfunc_end', i)
        body = s[i:j].split('\n')
        probs = (C.check(body, nm) + C.check_vmem(body, nm) + C.check_store_data(body, nm) + C.check_flat(body, nm) +
                 C.check_private(body, nm))
        if probs:
            bad.append('%s %s: %d (first: %s)' % (tu, nm, len(probs), probs[0][1]))
        if any(re.fullmatch(pat, nm) for pat in LOOP_WAIT_FREE.get(tu, [])):
            loops[nm] = tile_loop_vmcnt_waits([ln.strip() for ln in body])
        if any(re.fullmatch(pat, nm) for pat in NT_STORE_KERNELS.get(tu, [])):
            st = [ln.strip() for ln in body if ln.strip().startswith('global_store_dwordx4')]
            plain[nm] = (len(st), [ln for ln in st if not re.search(r'\bnt\b', ln)])
    return bad, loops, plain


_RESULTS = {}


def _isa_results():
    """Every TU compiled and checked once per test session (the TUs compile in parallel; tu_w1 takes minutes)."""
    if not _RESULTS:
        from concurrent.futures import ProcessPoolExecutor
        with ProcessPoolExecutor(max_workers=min(8, os.cpu_count() or 2)) as ex:
            for tu, res in zip(TUS, ex.map(_compile_and_check, TUS)):
                _RESULTS[tu] = res
    return _RESULTS


@pytest.mark.skipif(shutil.which('hipcc') is None and not os.path.exists('/opt/rocm/bin/hipcc'),
                    reason='hipcc not available')
def test_no_read_of_inflight_lds_load_registers():
    bad = [b for tu in TUS for b in _isa_results()[tu][0]]
    assert not bad, '\n'.join(bad)


@pytest.mark.skipif(shutil.which('hipcc') is None and not os.path.exists('/opt/rocm/bin/hipcc'),
                    reason='hipcc not available')
def test_counted_tile_loops_have_no_compiler_vmcnt():
    """The recompute W2 store (the next tile's inputs as asm loads), the fp32 reverse (also the delta_0 tail's cos
    blocks prefetched at mid NS - 3, the next tile's first cos blocks at the last mid, a counted tile-start wait) and
    the split-bf16 reverse count every vector-memory operation of their tile loop themselves. A compiler s_waitcnt vmcnt there does not know the asm operations and drains the weight ring
    (a scratch reload, or a compiler load consumed at the next tile start)."""
    res = _isa_results()
    for tu, pats in LOOP_WAIT_FREE.items():
        loops = res[tu][1]
        assert len(loops) >= len(pats), (tu, sorted(loops))
        for nm, waits in loops.items():
            assert waits is not None, '%s: no tile loop found' % nm
            assert not waits, '%s: compiler vmcnt waits in the tile loop: %s' % (nm, waits)


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
def test_tile_stores_are_nontemporal():
    """The store-heavy kernels' 16-byte tile / kept-jet stores carry the nontemporal hint (SIREN_STORE_NT)."""
    res = _isa_results()
    for tu, pats in NT_STORE_KERNELS.items():
        plain = res[tu][2]
        assert plain, (tu, 'no kernel matched', pats)
        for nm, (n, bad) in plain.items():
            assert n > 0, '%s: no 16-byte stores found' % nm
            assert not bad, '%s: %d of %d stores without nt (first: %s)' % (nm, len(bad), n, bad[0])
