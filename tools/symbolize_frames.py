#!/usr/bin/env python3
"""Name the library and function of unsymbolized stack frames from a crash trace (glog-style
`@ 0x... (unknown)` lines) without the process's /proc/<pid>/maps.

Frames of one library keep their pairwise differences under ASLR (one load base), and every
frame but the faulting one is a return address: the instruction right after a `call`. For a
group of frames believed to share a library, every page-aligned base that puts ALL of them
just after call instructions of a candidate library is reported, with the function each frame
falls in (objdump's symbol for the enclosing function).

usage: tools/symbolize_frames.py <group: addr,addr,...> [<group> ...] -- <library> [<library> ...]
A group prefixed with `pc:` is a faulting PC (an instruction boundary, not a return address); inside a
group of return addresses one address may carry `pc:` itself (the PC with the frames near it).
"""
import bisect
import re
import subprocess
import sys

CALL = re.compile(r"^\s*([0-9a-f]+):\s+(call|callq)\b")
INSN = re.compile(r"^\s*([0-9a-f]+):\s")
FUNC = re.compile(r"^([0-9a-f]+) <(.+)>:$")


def disasm(lib):
    """(sorted return addresses, sorted instruction starts, sorted [(start, name)] functions)"""
    out = subprocess.run(["objdump", "-d", "--no-show-raw-insn", "-C", lib], capture_output=True, text=True,
                         check=True).stdout.splitlines()
    rets, insns, funcs = [], [], []
    pending_call = False
    for line in out:
        m = FUNC.match(line)
        if m:
            funcs.append((int(m.group(1), 16), m.group(2)))
            continue
        m = INSN.match(line)
        if not m:
            continue
        a = int(m.group(1), 16)
        insns.append(a)
        if pending_call:
            rets.append(a)
        pending_call = bool(CALL.match(line))
    return sorted(set(rets)), sorted(set(insns)), sorted(funcs)


def func_of(funcs, off):
    i = bisect.bisect_right(funcs, (off, chr(0x10FFFF))) - 1
    return funcs[i][1] if i >= 0 else "?"


def main():
    argv = sys.argv[1:]
    sep = argv.index("--")
    groups, libs = argv[:sep], argv[sep + 1:]
    for lib in libs:
        rets, insns, funcs = disasm(lib)
        rset, iset = set(rets), set(insns)
        for grp in groups:
            is_pc = grp.startswith("pc:")
            # a whole group prefixed pc: is faulting PCs; inside a group, one address prefixed pc:
            # is the faulting PC among return addresses (mixed: the PC and the frames near it)
            items = [x for x in grp[3 if is_pc else 0:].split(",")]
            kinds = [is_pc or x.startswith("pc:") for x in items]
            addrs = [int(x[3:] if x.startswith("pc:") else x, 16) for x in items]
            hits = []
            a0, k0 = addrs[0], kinds[0]
            for r in (insns if k0 else rets):
                if (r & 0xFFF) != (a0 & 0xFFF):
                    continue
                base = a0 - r
                if base & 0xFFF:
                    continue
                ok = all(((a - base) in (iset if k else rset)) for a, k in zip(addrs, kinds))
                if ok:
                    hits.append(base)
            label = ("pc " if is_pc else "") + ",".join(hex(a) for a in addrs)
            if not hits:
                print("%-40s %s: no base fits" % (lib.split("/")[-1], label))
                continue
            print("%-40s %s: %d base(s) fit" % (lib.split("/")[-1], label, len(hits)))
            for base in hits[:6]:
                print("    base %s" % hex(base))
                for a in addrs:
                    print("      %s = +%s  %s" % (hex(a), hex(a - base), func_of(funcs, a - base)[:150]))


if __name__ == "__main__":
    main()
