"""Static check of a kernel's ISA for reads of in-flight LDS-load destinations.

hipcc does not count inline-asm ds_read loads: their destination VGPRs count as written at the asm statement, so the
compiler may copy, spill or reuse them before the data lands (cdna_hip_programming.md 'What hipcc does not do').
This walks each kernel's ISA along its control-flow graph (fall-through labels and branch edges, loop back-edges
iterated to a fixed point), tracks the destinations of every ds_read in issue order and the
s_waitcnt lgkmcnt(N) that retires them (LDS loads complete in order), and reports any instruction that reads or
overwrites a register of a load that is still outstanding.

python tools/check_asm_waits.py <file.s> [kernel-substring]   (hipcc --cuda-device-only -S output)
"""
import functools
import re
import sys

REG = re.compile(r'\b([va])(\d+)\b|\b([va])\[(\d+):(\d+)\]')


@functools.lru_cache(maxsize=None)
def regs(text):
    out = set()
    for m in REG.finditer(text):
        if m.group(1):
            out.add((m.group(1), int(m.group(2))))
        else:
            for r in range(int(m.group(4)), int(m.group(5)) + 1):
                out.add((m.group(3), r))
    return frozenset(out)


BRANCH = re.compile(r'^(s_branch|s_cbranch_\w+)\s+(\S+)')
TERMINAL = ('s_branch', 's_endpgm', 's_setpc_b64')


def _merge(a, b):
    """Join two outstanding-load lists at a control-flow merge: the loads complete in order and a wait keeps the
    N youngest, so align the lists at their young end and union the registers position by position (the longer
    list's older entries are kept). Sound for any wait either path reaches the join with."""
    if a is None or b is None:
        return list(a if b is None else b)
    n = max(len(a), len(b))
    out = []
    for k in range(n, 0, -1):
        ea = a[len(a) - k] if k <= len(a) else None
        eb = b[len(b) - k] if k <= len(b) else None
        if ea is None:
            out.append(eb)
        elif eb is None:
            out.append(ea)
        else:
            out.append((min(ea[0], eb[0]), ea[1] | eb[1]))
    return _trim(out)


def _trim(pending):
    """Drop the oldest entries that hold no register (stores, LDS-DMA loads, writes): only the positions of the
    register-holding loads relative to the young end matter, so this is the canonical form the fixed point needs."""
    k = 0
    while k < len(pending) and not pending[k][1]:
        k += 1
    return pending[k:] if k else pending


SREG = re.compile(r'\bs(\d+)\b|\bs\[(\d+):(\d+)\]')


@functools.lru_cache(maxsize=None)
def _sregs(text):
    out = set()
    for m in SREG.finditer(text):
        if m.group(1):
            out.add(int(m.group(1)))
        else:
            out.update(range(int(m.group(2)), int(m.group(3)) + 1))
    return frozenset(out)


def _facts_after(t, op, facts, tracked=None):
    """Branch-condition facts after instruction t. hipcc lowers `if (c) wait_a; else wait_b;` (and a condition
    tested twice, like `if (more) issue loads` ... `if (more) wait(4) else wait(0)`) into separate branches on a
    uniform mask it keeps in an SGPR pair, so without these facts the walk takes paths that skip every wait (an
    infeasible one) and reports a false race. Tracked: SGPR pairs known zero / non-zero (s_mov_b64 of an immediate,
    or learnt from a branch on vcc computed from them) and vcc as `s_and(n2)_b64 vcc, exec, s[..]` of such a pair
    (uniform masks: exec & s is zero iff s is zero in a running wave). Any other write of a tracked register, or any
    other write of vcc, forgets what depended on it (conservative)."""
    if 'vcc' not in t and not op.startswith('s_'):
        return facts
    f = dict(facts)
    ops = [x.strip() for x in t[len(op):].split(',')]
    dst = ops[0] if ops else ''
    if op.startswith('s_cbranch') or op in ('s_waitcnt', 's_barrier', 's_nop') or op.startswith('s_load') or \
            op.startswith('s_buffer_load') or op.startswith('s_set') or op.startswith('s_sleep'):
        if op.startswith('s_load') or op.startswith('s_buffer_load'):
            pass  # falls through to the register-write rule below
        else:
            return facts
    if dst == 'vcc':
        f.pop('vcc', None)
        if op in ('s_and_b64', 's_andn2_b64') and len(ops) == 3 and ops[1] == 'exec':
            src = _sregs(ops[2])
            neg = op == 's_andn2_b64'
            if src in f:
                v = f[src]
                f['vcc'] = v if not neg else ('z' if v == 'nz' else 'nz')
            elif src:
                f['vcc'] = ('src', src, neg)
        return tuple(sorted(f.items(), key=str))
    if 'vcc' in t and op.startswith('v_') and ('vcc' in dst or (len(ops) > 1 and ops[1] == 'vcc' and '_co' in op)):
        f.pop('vcc', None)  # v_cmp_*_e32 / carry-out writes
        return tuple(sorted(f.items(), key=str))
    if op.startswith('s_'):
        w = _sregs(dst)
        if w:
            for k in [k for k in f if k != 'vcc' and k & w]:
                f.pop(k)
            vc = f.get('vcc')
            if isinstance(vc, tuple) and vc[1] & w:
                f.pop('vcc')
            if op == 's_mov_b64' and len(ops) == 2 and (tracked is None or w in tracked):
                try:
                    f[w] = 'z' if int(ops[1], 0) == 0 else 'nz'
                except ValueError:
                    pass
    return tuple(sorted(f.items(), key=str))


def _edges(op, facts):
    """[(feasible, facts on that edge)] for the taken and the fall-through edge of a conditional branch."""
    f = dict(facts)
    vc = f.get('vcc')
    if op not in ('s_cbranch_vccz', 's_cbranch_vccnz'):
        return (True, facts), (True, facts)
    res = []
    for taken in (True, False):
        v = 'z' if (op == 's_cbranch_vccz') == taken else 'nz'
        if vc in ('z', 'nz'):
            res.append((vc == v, facts))
            continue
        g = dict(f)
        g['vcc'] = v
        if isinstance(vc, tuple):
            _, src, neg = vc
            g[src] = v if not neg else ('z' if v == 'nz' else 'nz')
        res.append((True, tuple(sorted(g.items(), key=str))))
    return res[0], res[1]


def _join(states, facts, pending, limit=4):
    """Add one (facts, pending) path state into the dict of states at a program point; too many distinct fact
    sets collapse into the fact-free state."""
    out = dict(states)
    out[facts] = _merge(out.get(facts), pending)
    if len(out) > limit:
        acc = None
        for pd in out.values():
            acc = _merge(acc, pd)
        out = {(): acc}
    return out


def _walk(body, step, cap):
    """Run step(no, text, op, operands, pending, problems) -> pending over the kernel's control-flow graph: the
    outstanding-load list flows through fall-through labels and along every feasible s_branch / s_cbranch edge
    (loop back-edges included) until it stops changing, so a load still in flight at a label or a branch is checked
    at the target. Path states are kept apart by the branch facts of _facts_after. Problems are those of the final
    pass (deduplicated)."""
    labels = set()
    tracked = set()  # SGPR pairs some branch condition is computed from: the only ones worth a fact
    for line in body:
        t = line.split(';')[0].strip()
        if t.endswith(':'):
            labels.add(t[:-1])
        elif t.startswith('s_and') and t.split(',')[0].endswith('vcc') and ' exec,' in t:
            tracked.add(_sregs(t.split(',')[-1].strip()))
    at_label = {}
    collapsed = set()
    for _ in range(24):
        changed = False
        problems = []
        cur = {(): []}  # facts -> pending; empty dict = unreachable by fall-through
        for no, line in enumerate(body):
            t = line.split(';')[0].strip()
            if not t or t.startswith('.') and not t.endswith(':'):
                continue
            if t.endswith(':'):
                for fx, pd in at_label.get(t[:-1], {}).items():
                    cur = _join(cur, fx, pd)
                continue
            if not cur:
                continue
            op = t.split()[0]
            m = BRANCH.match(t)
            if m and m.group(2) in labels:
                tgt = m.group(2)
                nxt = {}
                for fx, pd in cur.items():
                    (take, ft), (fall, ff) = _edges(op, fx) if op != 's_branch' else ((True, fx), (False, fx))
                    if take:
                        old = at_label.get(tgt, {})
                        new = _join(old, () if tgt in collapsed else ft, pd)
                        if len(new) == 1 and () in new and len(old) + (ft not in old) > 1:
                            collapsed.add(tgt)  # sticky: a label that once held too many fact sets stays fact-free
                        if new != old:
                            at_label[tgt] = new
                            changed = True
                    if fall:
                        nxt = _join(nxt, ff, pd)
                cur = nxt
                continue
            if op in TERMINAL:
                cur = {}
                continue
            nxt = {}
            for fx, pd in cur.items():
                pd = step(no, t, op, t[len(op):], pd, problems)
                if len(pd) > cap:  # the counter saturates: issue stalls until the oldest completes
                    pd = _trim(pd[len(pd) - cap:])
                elif pd and not pd[0][1]:
                    pd = _trim(pd)
                nxt = _join(nxt, _facts_after(t, op, fx, tracked), pd)
            cur = nxt
        if not changed:
            break
    seen, out = set(), []
    for p in problems:
        if p[0] not in seen:
            seen.add(p[0])
            out.append(p)
    return out


def _lgkm_step(no, t, op, operands, pending, problems):
    if op == 's_waitcnt':
        m = re.search(r'lgkmcnt\((\d+)\)', t)
        if m:
            keep = int(m.group(1))
            pending = [] if keep == 0 else pending[len(pending) - keep:] if keep < len(pending) else pending
        return pending
    if op.startswith('s_load') or op.startswith('s_buffer_load'):
        return pending + [(no, set())]  # counted in lgkmcnt too
    if op.startswith('s_') and 'barrier' not in op:
        return pending
    if op.startswith('ds_') and not op.startswith('ds_read'):
        used = regs(operands)
        for ln, rs in pending:
            if rs & used:
                problems.append((no, t, ln))
        return pending + [(no, set())]  # LDS writes / other LDS ops count in lgkmcnt
    if op.startswith('ds_read'):
        parts = operands.split(',')
        dst = regs(parts[0])
        src = regs(','.join(parts[1:]))
        for ln, rs in pending:
            if rs & (dst | src):
                problems.append((no, t, ln))
        return pending + [(no, dst)]
    used = regs(operands)
    for ln, rs in pending:
        if rs & used:
            problems.append((no, t, ln))
    return pending


def check(body, name):
    """Reads / overwrites of in-flight LDS-load destinations (lgkmcnt)."""
    return _walk(body, _lgkm_step, 15)  # lgkmcnt is 4 bits


VMEM = ('global_', 'buffer_', 'scratch_')


def _vmem_step(no, t, op, operands, pending, problems):
    if op == 's_waitcnt':
        m = re.search(r'vmcnt\((\d+)\)', t)
        if m:
            keep = int(m.group(1))
            pending = [] if keep == 0 else pending[len(pending) - keep:] if keep < len(pending) else pending
        return pending
    if op.startswith('s_'):
        return pending
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
        return pending + [(no, dst)]
    used = regs(operands)
    for ln, rs in pending:
        if rs & used:
            problems.append((no, t, ln))
    return pending


def check_vmem(body, name):
    """The same walk for vector-memory loads (the saddr-form asm loads of w1_kernel's REV cos prefetch and
    w3i_kernel's epilogue reloads): every global_/buffer_/scratch_ op counts in vmcnt in issue order (stores and
    LDS-DMA loads too, with no register destination), s_waitcnt vmcnt(N) keeps the N youngest outstanding, and an
    instruction that touches a load's destination before the wait that retires it is reported."""
    return _walk(body, _vmem_step, 63)  # vmcnt is 6 bits


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


def check_flat(body, name):
    """FLAT memory instructions (flat_load / flat_store / flat_atomic): hipcc emits them for a generic pointer whose
    address space it cannot prove (one stepped through an opaque asm register). A FLAT op counts in lgkmcnt as well
    as vmcnt and may retire out of order with the LDS reads there, so every counted `s_waitcnt lgkmcnt(N)` of the
    MFMA operand prefetch behind it is both slow (it waits for the store to reach memory) and not a valid wait for
    the LDS read it guards. Every kernel here addresses global memory through global_ ops (siren_common.h gmem)."""
    problems = []
    for no, line in enumerate(body):
        t = line.split(';')[0].strip()
        if t.startswith('flat_'):
            problems.append((no, t, None))
    return problems


def check_private(body, name):
    """Explicit private-memory (scratch) accesses — a context struct or array the compiler could not keep in registers
    (SROA blocked, e.g. by a scalar field's splat widened into a 16-byte load), whose fields are then reloaded from
    scratch with a vmcnt wait in the hot loop. Register spills ("Folded Spill / Reload") are not reported here."""
    problems = []
    for no, line in enumerate(body):
        t = line.strip()
        if t.startswith('scratch_') and 'Folded' not in t:
            problems.append((no, t.split(';')[0].strip(), None))
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
        probs = (check(body, nm) + check_vmem(body, nm) + check_store_data(body, nm) + check_flat(body, nm) +
                 check_private(body, nm))
        print('%-70s %d reads of in-flight load registers' % (nm[:70], len(probs)))
        for no, t, ln in probs[:8]:
            print('    line %d: %s   (load at line %d: %s)' % (no, t, ln, body[ln].strip()))
        bad += len(probs)
    sys.exit(1 if bad else 0)


if __name__ == '__main__':
    main()
