"""Materialises INTEGRATION.md's reference-side binding for compilation.

TEST INFRASTRUCTURE ONLY (oracle/ref/Makefile, target `adapter`). It reads
INTEGRATION.md and writes, under the output directory (oracle/_ref/adapter,
git-ignored, never shipped as source):

* every `<!-- adapter-file: PATH -->` block verbatim as PATH (the adapter header
  src/integrators/bdpt_gpu.h), and
* copies of the reference files that the `<!-- adapter-edit: FILE after|before
  "ANCHOR" -->` blocks edit (src/core/core.h, src/main.cpp,
  src/core/renderer.cpp) with each block inserted next to the one line of FILE
  whose stripped text equals ANCHOR (plus the edited files' unedited sibling
  headers, so relative includes resolve to one copy). An anchor that is missing
  or repeated is an error, so the document cannot drift from what the tests
  compile.

Usage: make_adapter.py INTEGRATION.md REFERENCE_ROOT OUT_DIR
"""
from __future__ import annotations

import json
import os
import re
import sys

MARK = re.compile(r'^<!-- adapter-(file|edit): (\S+)(?: (after|before) ("(?:[^"\\]|\\.)*"))? -->\s*$')


def blocks(doc: str):
    lines = doc.splitlines()
    i = 0
    while i < len(lines):
        m = MARK.match(lines[i])
        if not m:
            i += 1
            continue
        kind, path, where, anchor = m.group(1), m.group(2), m.group(3), m.group(4)
        j = i + 1
        if j >= len(lines) or not lines[j].startswith("```"):
            raise SystemExit(f"INTEGRATION.md:{i + 1}: marker not followed by a fenced block")
        k = j + 1
        while k < len(lines) and lines[k] != "```":
            k += 1
        if k >= len(lines):
            raise SystemExit(f"INTEGRATION.md:{j + 1}: unterminated fenced block")
        yield kind, path, where, (json.loads(anchor) if anchor else None), lines[j + 1:k], i + 1
        i = k + 1


def main(argv):
    if len(argv) != 4:
        raise SystemExit(__doc__)
    doc_path, ref, out = argv[1:]
    with open(doc_path) as f:
        doc = f.read()
    edited: dict[str, list[str]] = {}
    files = 0
    for kind, path, where, anchor, body, line in blocks(doc):
        if kind == "file":
            dst = os.path.join(out, path)
            os.makedirs(os.path.dirname(dst), exist_ok=True)
            with open(dst, "w") as f:
                f.write("\n".join(body) + "\n")
            files += 1
            continue
        if where is None:
            raise SystemExit(f"INTEGRATION.md:{line}: adapter-edit needs after|before \"ANCHOR\"")
        if path not in edited:
            with open(os.path.join(ref, path), encoding="utf-8", errors="surrogateescape") as f:
                edited[path] = f.read().split("\n")
        text = edited[path]
        hits = [n for n, t in enumerate(text) if t.strip() == anchor]
        if len(hits) != 1:
            raise SystemExit(f"INTEGRATION.md:{line}: anchor {anchor!r} found {len(hits)} times in {path}")
        at = hits[0] + (1 if where == "after" else 0)
        text[at:at] = body
    if files == 0 or not edited:
        raise SystemExit("INTEGRATION.md: no adapter-file / adapter-edit blocks found")
    for path, text in edited.items():
        dst = os.path.join(out, path)
        os.makedirs(os.path.dirname(dst), exist_ok=True)
        # the edited file's unedited sibling headers come along, so its quoted
        # includes ("platform.h", and "core.h" from accel.h) resolve to one copy
        src_dir = os.path.join(ref, os.path.dirname(path))
        for name in sorted(os.listdir(src_dir)):
            sib = os.path.join(os.path.dirname(path), name)
            if name.endswith(".h") and sib not in edited:
                with open(os.path.join(src_dir, name), "rb") as f, open(os.path.join(out, sib), "wb") as g:
                    g.write(f.read())
        with open(dst, "w", encoding="utf-8", errors="surrogateescape") as f:
            f.write("\n".join(text))
    print(f"adapter: {files} file(s), {len(edited)} edited reference file(s) -> {out}")


if __name__ == "__main__":
    main(sys.argv)
