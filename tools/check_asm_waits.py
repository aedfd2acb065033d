"""Static check of a kernel's ISA for reads of in-flight LDS-load destinations.

hipcc does not count inline-asm ds_read loads: their destination VGPRs count as written at the asm statement, so the
compiler may copy, spill or reuse them before the data lands (cdna_hip_programming.md 'What hipcc does not do').
This walks each kernel's straight-line ISA, tracks the destinations of every ds_read in issue order and the
s_waitcnt lgkmcnt(N) that retires them (LDS loads complete in order), and reports any instruction that reads or
overwrites a register of a load that is still outstanding.

python tools/check_asm_waits.py <file.s> [kernel-substring]   (hipcc --cuda-device-only -S output)
"""
import re
import sys

REG = re.compile(r'\b([va])(\d+)\b|\b([va])\[(\d+):(\d+)\]')


def regs(text):
    out = set()
    for m in REG.finditer(text):
        if m.group(1):
            out.add((m.group(1), int(m.group(2))))
        else:
            for r in range(int(m.group(4)), int(m.group(5)) + 1):
                out.add((m.group(3), r))
    return out


def check(body, name):
    pending = []  # list of (line_no, set of regs) for outstanding LDS loads, oldest first
    problems = []
    for no, line in enumerate(body):
        t = line.split(';')[0].strip()
        if not t or t.endswith(':') or t.startswith('.'):
            if t.endswith(':'):
                pending = []  # a label: control-flow join; be conservative and reset (loop heads wait themselves)
            continue
        op = t.split()[0]
        if op == 's_waitcnt':
            m = re.search(r'lgkmcnt\((\d+)\)', t)
            if m:
                keep = int(m.group(1))
                pending = pending[len(pending) - keep:] if keep < len(pending) else pending
                if keep == 0:
                    pending = []
            continue
        if op.startswith('s_load') or op.startswith('s_buffer_load'):
            pending.append((no, set()))  # counted in lgkmcnt too
            continue
        if op.startswith('s_') and 'barrier' not in op:
            continue
        operands = t[len(op):]
        if op.startswith('ds_') and not op.startswith('ds_read'):
            used = regs(operands)
            for ln, rs in pending:
                if rs & used:
                    problems.append((no, t, ln))
            pending.append((no, set()))  # LDS writes / other LDS ops count in lgkmcnt
            continue
        if op.startswith('ds_read'):
            parts = operands.split(',')
            dst = regs(parts[0])
            src = regs(','.join(parts[1:]))
            for ln, rs in pending:
                if rs & (dst | src):
                    problems.append((no, t, ln))
            pending.append((no, dst))
            continue
        used = regs(operands)
        for ln, rs in pending:
            if rs & used:
                problems.append((no, t, ln))
    return problems


VMEM = ('global_', 'buffer_', 'scratch_')


def check_vmem(body, name):
    """The same walk for vector-memory loads (the saddr-form asm loads of w1_kernel's REV cos prefetch and
    w3i_kernel's epilogue reloads): every global_/buffer_/scratch_ op counts in vmcnt in issue order (stores and
    LDS-DMA loads too, with no register destination), s_waitcnt vmcnt(N) keeps the N youngest outstanding, and an
    instruction that touches a load's destination before the wait that retires it is reported."""
    pending = []
    problems = []
    for no, line in enumerate(body):
        t = line.split(';')[0].strip()
        if not t or t.endswith(':') or t.startswith('.'):
            if t.endswith(':'):
                pending = []
            continue
        op = t.split()[0]
        if op == 's_waitcnt':
            m = re.search(r'vmcnt\((\d+)\)', t)
            if m:
                keep = int(m.group(1))
                pending = pending[len(pending) - keep:] if 0 < keep < len(pending) else ([] if keep == 0 else pending)
            continue
        if op.startswith('s_'):
            continue
        operands = t[len(op):]
        if op.startswith(VMEM):
            parts = operands.split(',')
            is_load = '_load' in op and '_lds' not in op
            dst = regs(parts[0]) if is_load else set()
            src = regs(','.join(parts[1:])) if is_load else regs(operands)
            for ln, rs in pending:
                # a later load may overwrite an in-flight load's destination (vector memory returns in order: hipcc
                # does this for partially used results); reading it as an address or as store data may not
                if rs & src:
                    problems.append((no, t, ln))
            pending.append((no, dst))
            continue
        used = regs(operands)
        for ln, rs in pending:
            if rs & used:
                problems.append((no, t, ln))
    return problems


def check_store_data(body, name, wait_states=2):
    """gfx940+ store-data hazard: a VALU (or v_accvgpr / v_mfma) may not write a data VGPR of a preceding
    global_/buffer_/scratch_ store wider than 64 bits within two wait states (the store reads its data late). hipcc
    pads its own stores; inline-asm stores are invisible to it, so they must carry the s_nop themselves."""
    problems = []
    recent = []  # (line, data regs, wait states still needed)
    for no, line in enumerate(body):
        t = line.split(';')[0].strip()
        if not t or t.startswith('.') or t.endswith(':'):
            continue
        op = t.split()[0]
        operands = t[len(op):]
        if op == 's_nop':
            n = int(operands.strip() or '0', 0) + 1
            recent = [(ln, rs, w - n) for ln, rs, w in recent if w - n > 0]
            continue
        if op.startswith('v_'):
            dst = regs(operands.split(',')[0])
            for ln, rs, w in recent:
                if rs & dst:
                    problems.append((no, t, ln))
        if op.startswith(VMEM) and '_store_dwordx' in op and op[-1] in '34':
            parts = operands.split(',')
            data = regs(parts[1]) if len(parts) > 1 else set()
            recent = [(ln, rs, w - 1) for ln, rs, w in recent if w - 1 > 0]
            recent.append((no, data, wait_states))
            continue
        recent = [(ln, rs, w - 1) for ln, rs, w in recent if w - 1 > 0]
    return problems


def main():
    path = sys.argv[1]
    want = sys.argv[2] if len(sys.argv) > 2 else ''
    s = open(path).read()
    names = re.findall(r'\n(_Z\w+):', s)
    bad = 0
    for nm in names:
        if want and want not in nm:
            continue
        i = s.find('\n' + nm + ':')
        j = s.find('.Lfunc_end', i)
        body = s[i:j].split('\n')
        probs = check(body, nm) + check_vmem(body, nm) + check_store_data(body, nm)
        print('%-70s %d reads of in-flight load registers' % (nm[:70], len(probs)))
        for no, t, ln in probs[:8]:
            print('    line %d: %s   (load at line %d: %s)' % (no, t, ln, body[ln].strip()))
        bad += len(probs)
    sys.exit(1 if bad else 0)


if __name__ == '__main__':
    main()
