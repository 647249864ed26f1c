#!/usr/bin/env python3
"""Audit of uncounted asm loads (mph_kernels.hip start_load) in a gfx950 assembly listing: from
every `buffer_load_dword vN ... offen` between ;;#ASMSTART/;;#ASMEND, walk every control-flow path
until an `s_waitcnt vmcnt(0)`; any other instruction that names vN on the way reads (or copies,
or overwrites) the register before the load has landed -- a bug (cdna_hip_programming.md 5.7).

  python tools/asm_load_audit.py kernels.s [symbol-substring ...]
Exit status 1 if a violation is found.
"""
import re
import sys


def functions(text):
    out = {}
    cur = None
    for ln in text.splitlines():
        m = re.match(r'^(_Z\S+):', ln)
        if m:
            cur = m.group(1)
            out[cur] = []
            continue
        if cur is not None:
            if ln.startswith('.Lfunc_end'):
                cur = None
                continue
            out[cur].append(ln)
    return out


def audit(name, lines):
    # instructions (stripped, no comments) with label positions
    ins, labels = [], {}
    for ln in lines:
        s = ln.split(';')[0].strip() if not ln.strip().startswith(';;#ASM') else ln.strip()
        if not s:
            continue
        m = re.match(r'^(\.LBB\S+):', s)
        if m:
            labels[m.group(1)] = len(ins)
            continue
        if s.startswith('.'):
            continue
        ins.append(s)
    bad = []
    for i, s in enumerate(ins):
        m = re.match(r'buffer_load_dword (v\d+), v\d+, s\[\d+:\d+\], 0 offen$', s)
        if not m or i == 0 or ins[i - 1] != ';;#ASMSTART':
            continue
        reg = m.group(1)
        pat = re.compile(r'(?<![\w\[:])' + reg + r'(?![\w\]:])|v\[(\d+):(\d+)\]')
        regn = int(reg[1:])
        seen = set()
        stack = [i + 1]
        while stack:
            k = stack.pop()
            while k < len(ins):
                if k in seen:
                    break
                seen.add(k)
                t = ins[k]
                if t.startswith('s_waitcnt') and 'vmcnt(0)' in t:
                    break
                if not t.startswith(';;#ASM'):
                    hit = False
                    for mm in pat.finditer(t):
                        if mm.group(1) is None or int(mm.group(1)) <= regn <= int(mm.group(2)):
                            hit = True
                    if hit:
                        bad.append((reg, i, k, t))
                        break
                op = t.split()[0]
                if op == 's_branch':
                    k = labels[t.split()[1]]
                    continue
                if op.startswith('s_cbranch'):
                    stack.append(labels[t.split()[1]])
                if op in ('s_endpgm', 's_setpc_b64'):
                    break
                k += 1
    return bad


def main():
    text = open(sys.argv[1]).read()
    keys = sys.argv[2:] or ['k_neighbors']
    rc = 0
    nfun = 0
    for name, lines in functions(text).items():
        if not any(k in name for k in keys):
            continue
        nfun += 1
        for reg, i, k, t in audit(name, lines):
            print('%s: %s loaded at instr %d is used at %d before vmcnt(0): %s' % (name[:60], reg, i, k, t))
            rc = 1
    print('audited %d functions: %s' % (nfun, 'VIOLATIONS' if rc else 'clean'))
    return rc


if __name__ == '__main__':
    sys.exit(main())
