#!/usr/bin/env python3
"""Remove preprocessor conditionals on the given macros, taking them as undefined.

    python tools/unifdef.py FILE... -U RP_A -U RP_B

Only conditions of the forms `#ifdef M`, `#ifndef M`, `#if defined(M)`,
`#if !defined(M)` (and the `#elif` forms) on the listed macros are resolved; any
other conditional is kept verbatim. Used to strip measured-and-rejected A/B
variants out of the kernel sources.
"""
import argparse
import re
import sys

DIR = re.compile(r"^\s*#\s*(ifdef|ifndef|if|elif|else|endif)\b\s*(.*?)\s*(//.*)?$")
DEF = re.compile(r"^(!?)\s*defined\s*\(?\s*(\w+)\s*\)?$")


def cond_value(kind, expr, undef):
    """True/False if resolvable under `undef`, else None."""
    if kind == "ifdef":
        return False if expr in undef else None
    if kind == "ifndef":
        return True if expr in undef else None
    m = DEF.match(expr)
    if not m or m.group(2) not in undef:
        return None
    return bool(m.group(1))


def process(lines, undef):
    out = []
    stack = []   # frames: [resolved, active, taken, parent_active]
    active = True
    for ln in lines:
        m = DIR.match(ln)
        if not m:
            if active:
                out.append(ln)
            continue
        kind, expr = m.group(1), m.group(2)
        if kind in ("ifdef", "ifndef", "if"):
            v = cond_value(kind, expr, undef)
            if v is None:
                stack.append([False, active, False, active])
                if active:
                    out.append(ln)
            else:
                stack.append([True, active and v, v, active])
                active = active and v
        elif kind == "elif":
            fr = stack[-1]
            v = cond_value("if", expr, undef)
            if not fr[0]:
                if v is not None:
                    raise SystemExit(f"resolvable #elif in an unresolved chain: {ln!r}")
                if fr[3]:
                    out.append(ln)
                continue
            if v is None:
                raise SystemExit(f"unresolvable #elif in a resolved chain: {ln!r}")
            take = (not fr[2]) and v
            fr[2] = fr[2] or v
            active = fr[3] and take
        elif kind == "else":
            fr = stack[-1]
            if not fr[0]:
                if fr[3]:
                    out.append(ln)
                continue
            active = fr[3] and not fr[2]
            fr[2] = True
        else:   # endif
            fr = stack.pop()
            if not fr[0] and fr[3]:
                out.append(ln)
            active = fr[3]
    if stack:
        raise SystemExit("unbalanced conditionals")
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("files", nargs="+")
    ap.add_argument("-U", action="append", default=[])
    a = ap.parse_args()
    for f in a.files:
        with open(f) as fh:
            lines = fh.readlines()
        new = process(lines, set(a.U))
        if new != lines:
            with open(f, "w") as fh:
                fh.writelines(new)
            print(f"{f}: {len(lines)} -> {len(new)} lines", file=sys.stderr)


if __name__ == "__main__":
    main()
