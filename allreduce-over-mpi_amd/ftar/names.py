"""Kernel-name handling shared by bench.py and tools/pmc_summary.py (no library load)."""


def kernel_symbol(name):
    """A kernel name as rocprofv3 prints it ("void ftar::(anonymous namespace)::reduce_lds_kernel<ftar::
    (anonymous namespace)::F32Sum, 2, 1, 2, 2, true>(ftar::(anonymous namespace)::Srcs<2>, ...)") reduced to
    its template id ("reduce_lds_kernel<F32Sum, 2, 1, 2, 2, true>"): the key that ties a PMC summary entry to
    the kernel a run launched (profiles/pmc_summary.json, bench.py)."""
    s = name.replace("ftar::(anonymous namespace)::", "").replace("(anonymous namespace)::", "")
    if s.startswith("void "):
        s = s[5:]
    depth = 0   # cut the parameter list: the first '(' outside template brackets
    for i, ch in enumerate(s):
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            return s[:i].strip()
    return s.strip()
