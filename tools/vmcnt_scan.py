"""List the compiler-emitted s_waitcnt vmcnt waits inside each kernel's last loop (the persistent tile loop).

The counted kernels (w1_kernel, w1x_kernel, ...) wait on their inline-asm loads and stores themselves; a wait the
compiler emits does not know those operations, so inside the tile loop it drains the weight ring (a scratch reload,
or a compiler load consumed at the next tile start, both produce one). Waits inside ;;#ASMSTART / ;;#ASMEND blocks
are the kernels' own and are skipped.

python tools/vmcnt_scan.py <file.s> [kernel-substring]   (hipcc --cuda-device-only -S output)
"""
import re
import sys


def scan(text, sub=''):
    out = {}
    for nm in re.findall(r'\n(_Z\w+):', text):
        if sub not in nm:
            continue
        i = text.find('\n' + nm + ':')
        body = [ln.strip() for ln in text[i:text.find('.Lfunc_end', i)].split('\n')]
        headers = [k for k, ln in enumerate(body) if 'Loop Header' in ln]
        if not headers:
            continue
        in_asm, waits = False, []
        for k, ln in enumerate(body):
            if ln.startswith(';;#ASMSTART'):
                in_asm = True
            elif ln.startswith(';;#ASMEND'):
                in_asm = False
            elif not in_asm and k > headers[-1] and ln.startswith('s_waitcnt') and 'vmcnt' in ln:
                prev = next((body[q] for q in range(k - 1, max(k - 40, 0), -1)
                             if body[q] and not body[q].startswith(';') and 'load' in body[q]), '')
                waits.append((k, ln, prev))
        out[nm] = waits
    return out


def main():
    text = open(sys.argv[1]).read()
    for nm, waits in scan(text, sys.argv[2] if len(sys.argv) > 2 else '').items():
        print('%-70s %d compiler vmcnt waits in the tile loop' % (nm[:70], len(waits)))
        for k, ln, prev in waits[:8]:
            print('    line %d: %s   (last load before it: %s)' % (k, ln, prev[:60]))


if __name__ == '__main__':
    main()
