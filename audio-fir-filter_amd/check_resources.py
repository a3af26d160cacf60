"""Build-time check of liblcfir's kernel resources (Makefile, tests/test_build_resources.py).

fir_fft32r_kernel waits for its LDS-DMA with an explicit s_waitcnt
vmcnt(kR32PairStores) at the next unit's top (csrc/fir_fft32r.hpp): correct
only while the vector-memory instructions issued after the DMA are exactly the
pair stores.  A scratch spill or reload is a vector-memory instruction the
source cannot see, so every instance of that kernel must use no scratch.

usage: python3 check_resources.py REMARKS_FILE
(REMARKS_FILE: hipcc's stderr under -Rpass-analysis=kernel-resource-usage)
"""
import re
import sys

# kernels whose correctness depends on having no scratch accesses
NO_SCRATCH = ("fir_fft32r_kernel",)


def parse(text: str) -> dict:
    """{mangled kernel name: {field: int}} from kernel-resource-usage remarks."""
    out, cur = {}, None
    for line in text.splitlines():
        m = re.search(r"remark: Function Name: (\S+)", line)
        if m:
            cur = out.setdefault(m.group(1), {})
            continue
        m = re.search(r"remark:\s+([A-Za-z ]+?)(?: \[[^\]]*\])?: (\d+) \[-Rpass-analysis", line)
        if m and cur is not None:
            cur[m.group(1).strip()] = int(m.group(2))
    return out


def violations(kernels: dict) -> list:
    bad = []
    for name, f in kernels.items():
        if any(k in name for k in NO_SCRATCH):
            if f.get("ScratchSize", 0) or f.get("VGPRs Spill", 0):
                bad.append(f"{name}: ScratchSize {f.get('ScratchSize')} B/lane, "
                           f"VGPRs Spill {f.get('VGPRs Spill')}")
    return bad


def main(path: str) -> int:
    text = open(path).read()
    # pass the compiler's other diagnostics (warnings) through
    for line in text.splitlines():
        if "-Rpass-analysis=kernel-resource-usage" not in line and "remark:" not in line \
                and not re.match(r"^\s*(\d+ \|| *\||In file included)", line) and line.strip():
            print(line, file=sys.stderr)
    kernels = parse(text)
    checked = [n for n in kernels if any(k in n for k in NO_SCRATCH)]
    if not checked:
        print(f"check_resources: no {NO_SCRATCH} kernel in {path}", file=sys.stderr)
        return 1
    bad = violations(kernels)
    for b in bad:
        print(f"check_resources: scratch in a no-scratch kernel (its vmcnt wait would be wrong): {b}",
              file=sys.stderr)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
