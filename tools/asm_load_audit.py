#!/usr/bin/env python3
"""Audit of uncounted asm loads (mph_kernels.hip start_load) in a gfx950 assembly listing: from
every `buffer_load_dword vN ... offen` between ;;#ASMSTART/;;#ASMEND, walk every control-flow path
until an `s_waitcnt vmcnt(0)`; any other instruction that names vN on the way reads (or copies,
or overwrites) the register before the load has landed -- a bug (cdna_hip_programming.md 5.7).
The walk is path-sensitive for the structurizer's flow flags: an SGPR pair set to -1 / 0 and then
AND-ed with exec into vcc decides the following s_cbranch_vccz / vccnz (exec is never 0 in the
wave-uniform column loop), so infeasible paths through those branches are not reported.
Exec-skip branches count as not taken (execz) / taken (execnz): the caller's waits sit in
wave-uniform code, where exec is never 0.

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
    inside = False
    for i, s in enumerate(ins):
        if s == ';;#ASMSTART':
            inside = True
        elif s == ';;#ASMEND':
            inside = False
        m = re.match(r'buffer_load_dword (v\d+), v\d+, s\[\d+:\d+\], 0 offen$', s)
        if not m or not inside:
            continue
        reg = m.group(1)
        pat = re.compile(r'(?<![\w\[:])' + reg + r'(?![\w\]:])|v\[(\d+):(\d+)\]')
        regn = int(reg[1:])
        seen = set()
        stack = [(i + 1, frozenset(), None)]
        while stack:
            k, known, vcc = stack.pop()
            while k < len(ins):
                key = (k, known, vcc)
                if key in seen:
                    break
                seen.add(key)
                t = ins[k]
                if t.startswith('s_waitcnt') and 'vmcnt(0)' in t:
                    break
                if not t.startswith(';;#ASM') and not (t.startswith('buffer_load_dword') and t.endswith('offen')
                                                        and not re.match(r'buffer_load_dword ' + reg + r',', t)):
                    hit = False
                    for mm in pat.finditer(t):
                        if mm.group(1) is None or int(mm.group(1)) <= regn <= int(mm.group(2)):
                            hit = True
                    if hit:
                        bad.append((reg, i, k, t))
                        break
                op = t.split()[0]
                # constant tracking of SGPR pairs set to -1 / 0 (the structurizer's flow flags) and of
                # vcc = exec & pair (exec is never 0 in the wave-uniform code of the column loop)
                ops = [x.strip() for x in t[len(op):].split(',')] if len(t) > len(op) else []
                dst = ops[0] if ops else None
                if op == 's_mov_b64' and len(ops) == 2 and ops[1] in ('-1', '0'):
                    known = frozenset([x for x in known if x[0] != dst] + [(dst, ops[1])])
                elif dst is not None and dst.startswith('s[') and not op.startswith(('s_cbranch', 's_branch', 's_cmp')):
                    known = frozenset(x for x in known if x[0] != dst)
                if op == 's_and_b64' and dst == 'vcc' and len(ops) == 3 and 'exec' in ops[1:]:
                    other = ops[2] if ops[1] == 'exec' else ops[1]
                    kv = dict(known).get(other)
                    vcc = 'nz' if kv == '-1' else ('z' if kv == '0' else None)
                elif op == 's_andn2_b64' and dst == 'vcc' and len(ops) == 3 and ops[1] == 'exec':
                    kv = dict(known).get(ops[2])   # vcc = exec & ~pair
                    vcc = 'z' if kv == '-1' else ('nz' if kv == '0' else None)
                elif dst == 'vcc' or (op.startswith('v_cmp') and 'vcc' in t.split()[1:2][0] if len(t.split()) > 1 else False):
                    vcc = None
                if op == 's_branch':
                    k = labels[t.split()[1]]
                    continue
                if op == 's_cbranch_execz':
                    k += 1
                    continue
                if op == 's_cbranch_execnz':
                    k = labels[t.split()[1]]
                    continue
                if op == 's_cbranch_vccz' and vcc is not None:
                    k = labels[t.split()[1]] if vcc == 'z' else k + 1
                    continue
                if op == 's_cbranch_vccnz' and vcc is not None:
                    k = labels[t.split()[1]] if vcc == 'nz' else k + 1
                    continue
                if op.startswith('s_cbranch'):
                    stack.append((labels[t.split()[1]], known, vcc))
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
