#!/usr/bin/env python3
"""Resolve preprocessor conditionals on a fixed set of macros (a small `unifdef`).

    python tools/unifdef.py FILE -D NAME=VALUE ... -U NAME ... [-o OUT]

Chains (#if/#ifdef/#ifndef ... #elif ... #else ... #endif) whose every condition uses only the given macros
(and integer literals) are replaced by the body of the branch taken; chains with any other macro stay as
they are (their bodies are still processed).  Used to strip measured-and-not-kept variants out of the
product sources (they stay in git history)."""
import argparse
import re
import sys

DIRECTIVE = re.compile(r"^\s*#\s*(if|ifdef|ifndef|elif|else|endif)\b(.*)$")


def evaluate(kind, expr, defs, undefs):
    """True / False, or None when the condition uses a macro outside defs / undefs."""
    expr = re.sub(r"//.*$", "", expr)
    expr = re.sub(r"/\*.*?\*/", "", expr).strip()
    if kind in ("ifdef", "ifndef"):
        name = expr.split()[0]
        if name in defs:
            v = True
        elif name in undefs:
            v = False
        else:
            return None
        return v if kind == "ifdef" else not v

    def dfn(m):
        n = m.group(1)
        if n in defs:
            return " 1 "
        if n in undefs:
            return " 0 "
        raise KeyError(n)
    try:
        e = re.sub(r"defined\s*\(\s*(\w+)\s*\)", dfn, expr)
        e = re.sub(r"defined\s+(\w+)", dfn, e)
    except KeyError:
        return None
    for name in re.findall(r"\b[A-Za-z_]\w*\b", e):
        if name not in defs and name not in undefs:
            return None
    e = re.sub(r"\b([A-Za-z_]\w*)\b", lambda m: "(%s)" % defs.get(m.group(1), "0"), e)
    e = e.replace("&&", " and ").replace("||", " or ")
    e = re.sub(r"!(?!=)", " not ", e)
    return bool(eval(e, {}, {}))


def process(lines, defs, undefs):
    out = []
    i = 0
    n = len(lines)

    def block(i, depth_out):
        """Process lines from i until an #elif/#else/#endif at this level; returns (i, lines)."""
        res = []
        while i < n:
            m = DIRECTIVE.match(lines[i])
            if m and m.group(1) in ("elif", "else", "endif"):
                return i, res
            if m and m.group(1) in ("if", "ifdef", "ifndef"):
                i, chain = do_chain(i)
                res.extend(chain)
                continue
            res.append(lines[i])
            i += 1
        return i, res

    def do_chain(i):
        # collect branches: list of (directive line, kind, expr, body lines)
        branches = []
        m = DIRECTIVE.match(lines[i])
        kind, expr = m.group(1), m.group(2)
        head = lines[i]
        i += 1
        while True:
            i, body = block(i, None)
            branches.append((head, kind, expr, body))
            if i >= n:
                raise SystemExit("unterminated conditional")
            m = DIRECTIVE.match(lines[i])
            k = m.group(1)
            if k == "endif":
                end = lines[i]
                i += 1
                break
            head, kind, expr = lines[i], k, m.group(2)
            i += 1
        vals = []
        for head, kind, expr, body in branches:
            if kind == "else":
                vals.append(True)
            else:
                vals.append(evaluate("if" if kind == "elif" else kind, expr, defs, undefs))
        if any(v is None for v in vals):
            res = []
            for head, kind, expr, body in branches:
                res.append(head)
                res.extend(body)
            res.append(end)
            return i, res
        for (head, kind, expr, body), v in zip(branches, vals):
            if v:
                return i, body
        return i, []

    i, out = block(0, None)
    if i != n:
        raise SystemExit("stray directive at line %d: %s" % (i + 1, lines[i]))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("file")
    ap.add_argument("-D", action="append", default=[])
    ap.add_argument("-U", action="append", default=[])
    ap.add_argument("-o")
    a = ap.parse_args()
    defs = {}
    for d in a.D:
        k, _, v = d.partition("=")
        defs[k] = v or "1"
    lines = open(a.file).read().split("\n")
    out = process(lines, defs, set(a.U))
    # collapse runs of more than one blank line left behind
    res = []
    for l in out:
        if l.strip() == "" and res and res[-1].strip() == "":
            continue
        res.append(l)
    open(a.o or a.file, "w").write("\n".join(res))


if __name__ == "__main__":
    main()
