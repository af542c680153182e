"""Checks on the gfx950 ISA of the inline-asm sites of a kernel (or of every kernel with --all):
  * no instruction reads or writes the registers an inline-asm load writes before a wait that
    covers the load (CFG reachability): the waitcnt pass does not see asm loads.  An `s_waitcnt
    vmcnt(N)` covers a load when at least N vector-memory instructions follow the load on the path
    to it (returns come in issue order), so software-pipelined sites -- loads for the next step
    still in flight across a wait for this step's -- are checked load by load;
  * no VALU write of an SGPR that an inline-asm vector-memory instruction reads comes within 5 wait
    states of it (the compiler's hazard recognizer does not look inside inline asm);
  * every inline-asm instruction is of a kind these checks cover (vector loads, `s_waitcnt`,
    `s_nop`, VALU SDWA ops on VGPRs): a new kind of asm site fails until it is classified.
usage: python tools/asm_inflight_check.py ISA.s KERNEL_SYMBOL_SUBSTRING
       python tools/asm_inflight_check.py --all ISA.s [ISA.s ...]"""
import re
import sys

# inline-asm instruction kinds the checks below cover
KNOWN = ("buffer_load", "global_load", "s_waitcnt", "s_nop", "v_and_b32_sdwa")


def kernels_with_asm(s):
    """Symbols of the functions in an ISA file that contain inline asm."""
    out = []
    for m in re.finditer(r'^(_\S+):\s*;\s*@', s, flags=re.M):
        start = m.end()
        end = s.index('.Lfunc_end', start)
        if ';;#ASMSTART' in s[start:end]:
            out.append(m.group(1))
    return out


def main(path, kname):
    return check(open(path).read(), kname)


def check(s, kname):
    name_line = [l for l in s.split('\n') if l.startswith('_') and kname in l and re.match(r'^\S+:', l)][0]
    name_line = name_line.split(':')[0] + ':'

    start = s.index('\n' + name_line) + 1
    end = s.index('.Lfunc_end', start)
    body = s[start:end].split('\n')
    # basic blocks
    labels, blocks = {}, []
    cur = []
    for k, l in enumerate(body):
        t = l.strip()
        m = re.match(r'^(\.LBB\d+_\d+):', t)
        if m or t.startswith('; %bb.'):
            if cur:
                blocks.append(cur)
            cur = [k]
            if m:
                labels[m.group(1)] = len(blocks)
        else:
            cur.append(k)
    blocks.append(cur)
    blk_of = {}
    for bi, b in enumerate(blocks):
        for k in b:
            blk_of[k] = bi

    def succs(bi):
        out = []
        last = None
        for k in blocks[bi]:
            t = body[k].strip()
            if t and not t.startswith(';') and not t.startswith('.'):
                last = t
        for k in blocks[bi]:
            m = re.search(r's_c?branch\w*\s+(\.LBB\d+_\d+)', body[k])
            if m:
                out.append(labels[m.group(1)])
        if not (last and (last.startswith('s_branch') or last.startswith('s_endpgm'))) and bi + 1 < len(blocks):
            out.append(bi + 1)
        return out

    def regs_in(t):
        r = set()
        for m in re.finditer(r'v\[(\d+):(\d+)\]', t):
            r |= set(range(int(m.group(1)), int(m.group(2)) + 1))
        for m in re.finditer(r'\bv(\d+)\b', t):
            r.add(int(m.group(1)))
        return r

    asm_loads, asm_waits, asm_any, unknown = [], {}, set(), []
    inside = False
    for k, l in enumerate(body):
        if ';;#ASMSTART' in l:
            inside = True
            continue
        if ';;#ASMEND' in l:
            inside = False
            continue
        if inside:
            t = l.strip()
            asm_any.add(k)
            if t and not t.startswith(';') and not t.startswith('.') and not t.startswith(KNOWN):
                print(f"line {k}: unclassified inline-asm instruction: {t[:80]}")
                unknown.append(k)
            if t.startswith('buffer_load') or t.startswith('global_load'):
                asm_loads.append(k)
            if t.startswith('s_waitcnt') and 'vmcnt' in t:
                asm_waits[k] = t
    # every vmcnt wait (asm or compiler) with its count
    vwait = {}
    for k, l in enumerate(body):
        m = re.match(r'\s*s_waitcnt\b.*\bvmcnt\((\d+)\)', l)
        if m:
            vwait[k] = int(m.group(1))
    vmem = re.compile(r'\s*(buffer|global|flat|scratch)_(load|store|atomic)')
    regs = set()
    for k in asm_loads:
        regs |= regs_in(body[k].split(',')[0])
    bad = len(unknown)
    for k0 in asm_loads:
        own = regs_in(body[k0].split(',')[0])
        seen = set()
        stack = [(blk_of[k0], k0 + 1, 0)]
        while stack:
            bi, startk, cnt = stack.pop()
            if (bi, startk, cnt) in seen:
                continue
            seen.add((bi, startk, cnt))
            stop = False
            for k in blocks[bi]:
                if k < startk:
                    continue
                t = body[k].strip()
                if k in vwait and cnt >= vwait[k]:
                    stop = True  # the load has landed
                    break
                if vmem.match(body[k]):
                    cnt = min(cnt + 1, 64)
                if not t or t.startswith(';') or t.startswith('.') or k in asm_any:
                    continue
                u = regs_in(t) & own
                if u:
                    bad += 1
                    if bad <= 20:
                        print(f"line {k}: {sorted(u)} {t[:100]}  (after asm load line {k0})")
            if not stop:
                for sb in succs(bi):
                    stack.append((sb, blocks[sb][0], cnt))
    # gfx9 hazard: a VALU write of an SGPR that a VMEM instruction reads needs 5 wait states; the
    # compiler's hazard recognizer may not look inside inline asm
    def sregs(t):
        r = set()
        for m in re.finditer(r's\[(\d+):(\d+)\]', t):
            r |= set(range(int(m.group(1)), int(m.group(2)) + 1))
        for m in re.finditer(r'\bs(\d+)\b', t):
            r.add(int(m.group(1)))
        return r
    for k in sorted(asm_any):
        t = body[k].strip()
        if not (t.startswith('buffer_') or t.startswith('global_')):
            continue
        used = sregs(t)
        waits, q = 0, k - 1
        while q >= 0 and waits < 5:
            u = body[q].strip()
            if u.startswith('.LBB') or u.startswith('; %bb'):
                break
            if u and not u.startswith(';') and not u.startswith('.'):
                op = u.split()[0]
                if op.startswith('v_') and u.split()[1].rstrip(',').startswith('s'):
                    if sregs(u.split(',')[0]) & used:
                        bad += 1
                        print(f"line {k}: VALU SGPR write at line {q} within {waits} wait states: {u[:80]}")
                m = re.match(r's_nop\s+(\d+)', u)
                waits += (int(m.group(1)) + 1) if m else 1
            q -= 1
    print(f"{kname[:60]}: {len(asm_any)} asm lines, {len(asm_loads)} asm loads, {len(asm_waits)} asm waits, "
          f"registers {sorted(regs)}: {'OK' if not bad else str(bad) + ' VIOLATIONS'}")
    return 1 if bad else 0


def check_all(paths):
    rc, n = 0, 0
    for p in paths:
        s = open(p).read()
        for k in kernels_with_asm(s):
            rc |= check(s, k)
            n += 1
    print(f"{n} functions with inline asm checked: {'OK' if rc == 0 else 'VIOLATIONS'}")
    return rc


if __name__ == '__main__':
    if sys.argv[1] == '--all':
        sys.exit(check_all(sys.argv[2:]))
    sys.exit(main(sys.argv[1], sys.argv[2]))
