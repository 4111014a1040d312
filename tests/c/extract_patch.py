#!/usr/bin/env python3
"""Cut INTEGRATION.md section 1's patch out of the document, as written.

The two ```c blocks whose first line is `/* src/mem_sampling.c */` and
`/* src/mem_analyzer.c */` become two translation units, each prefixed with
`#include "ref_stubs.h"` (the reference declarations the patch relies on:
tests/c/ref_stubs.h).  They are compiled separately, like the reference's
own files, so a symbol one file uses from the other must be declared the way
the patch declares it.

  extract_patch.py INTEGRATION.md OUT_DIR
writes OUT_DIR/patch_mem_sampling.c and OUT_DIR/patch_mem_analyzer.c."""
import os
import re
import sys

MARKERS = {"/* src/mem_sampling.c */": "patch_mem_sampling.c",
           "/* src/mem_analyzer.c */": "patch_mem_analyzer.c"}


def extract(md_text):
    """{file name: block text} for the section-1 blocks (the first block per marker)."""
    out = {}
    for m in re.finditer(r"```c\n(.*?)```", md_text, re.S):
        body = m.group(1)
        first = body.split("\n", 1)[0].strip()
        name = MARKERS.get(first)
        if name and name not in out:
            out[name] = body
    missing = [n for n in MARKERS.values() if n not in out]
    if missing:
        raise SystemExit(f"extract_patch: no block for {missing} in INTEGRATION.md")
    return out


def main():
    md, outdir = sys.argv[1], sys.argv[2]
    os.makedirs(outdir, exist_ok=True)
    for name, body in extract(open(md).read()).items():
        text = f'/* generated from {os.path.basename(md)} by tests/c/extract_patch.py */\n#include "ref_stubs.h"\n' + body
        path = os.path.join(outdir, name)
        if not os.path.exists(path) or open(path).read() != text:
            with open(path, "w") as f:
                f.write(text)


if __name__ == "__main__":
    main()
