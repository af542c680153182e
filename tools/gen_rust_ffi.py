"""Print the Rust `extern "C"` block for every function of include/lsmblk.h.

Mechanical C -> Rust type mapping, so the binding a maintainer pastes into the reference crate
covers the whole ABI; tests/test_host_api.py checks INTEGRATION.md names every header symbol."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STRUCTS = {"lsmblk_builder": "LsmblkBuilder", "lsmblk_block": "LsmblkBlock", "lsmblk_iter": "LsmblkIter",
           "lsmblk_ctx": "LsmblkCtx", "lsmblk_kv_stream": "LsmblkKvStream", "lsmblk_compact_opts": "LsmblkCompactOpts",
           "lsmblk_key_range": "LsmblkKeyRange", "lsmblk_memtable": "LsmblkMemtable",
           "lsmblk_kernel_stat": "LsmblkKernelStat"}
SCALARS = {"int": "c_int", "uint32_t": "u32", "uint64_t": "u64", "size_t": "usize", "uint8_t": "u8",
           "uint16_t": "u16", "float": "f32", "char": "c_char", "void": "c_void", "int32_t": "i32"}


def rust_type(c):
    c = " ".join(c.replace("*", " * ").split())
    stars = c.count("*")
    base = c.replace("*", "").strip()
    const = base.startswith("const ")
    base = base.replace("const ", "").strip()
    t = STRUCTS.get(base) or SCALARS[base]
    if stars == 0:
        return t
    inner = ("*const " if const else "*mut ") + t
    for _ in range(stars - 1):
        inner = "*mut " + inner
    return inner


def functions():
    s = open(os.path.join(ROOT, "include", "lsmblk.h")).read()
    s = re.sub(r"/\*.*?\*/", "", s, flags=re.S)
    for m in re.finditer(r"^([a-z_0-9* ]+?)\b(lsmblk_[a-z0-9_]+)\s*\(([^;]*?)\);", s, flags=re.M | re.S):
        ret, name, args = m.group(1).strip(), m.group(2), " ".join(m.group(3).split())
        params = []
        if args != "void":
            for a in args.split(","):
                a = a.strip()
                mm = re.match(r"(.*?)([A-Za-z_][A-Za-z_0-9]*)$", a)
                ty, pn = mm.group(1).strip(), mm.group(2)
                if pn in ("in", "out", "ref", "type", "loop", "match"):
                    pn = pn + "_"
                params.append(f"{pn}: {rust_type(ty)}")
        r = "" if ret == "void" else " -> " + rust_type(ret)
        yield name, f"    pub fn {name}({', '.join(params)}){r};"


def splice(doc):
    """INTEGRATION.md with its extern block replaced by the current header's functions."""
    head, rest = doc.split('extern "C" {\n', 1)
    _, tail = rest.split("\n}\n", 1)
    body = "\n".join(line for _, line in functions())
    return head + 'extern "C" {\n' + body + "\n}\n" + tail


if __name__ == "__main__":
    import sys
    if "--write" in sys.argv:
        p = os.path.join(ROOT, "INTEGRATION.md")
        doc = splice(open(p).read())
        open(p, "w").write(doc)
    else:
        for _, line in functions():
            print(line)
