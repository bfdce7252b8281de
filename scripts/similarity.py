#!/usr/bin/env python
"""Share of a file's normalised code lines that also occur in a reference file.

Docstrings, comments and blank lines are dropped and whitespace is collapsed
before comparing; the ratio is |repo lines found in ref| / |repo lines|.

    python scripts/similarity.py REPO_FILE REF_FILE [REPO_FILE REF_FILE ...]
"""
import ast
import io
import re
import sys
import tokenize


def code_lines(path):
    src = open(path, encoding='utf-8').read()
    drop = set()
    try:
        tree = ast.parse(src)
        for node in ast.walk(tree):
            body = getattr(node, 'body', None)
            if isinstance(body, list) and body and isinstance(body[0], ast.Expr) and \
                    isinstance(getattr(body[0], 'value', None), ast.Constant) and isinstance(body[0].value.value, str):
                drop.update(range(body[0].lineno, body[0].end_lineno + 1))
    except SyntaxError:
        pass
    out = []
    toks = []
    try:
        toks = list(tokenize.generate_tokens(io.StringIO(src).readline))
    except (tokenize.TokenError, IndentationError):
        pass
    comment_lines = {t.start[0]: t.start[1] for t in toks if t.type == tokenize.COMMENT}
    for i, line in enumerate(src.splitlines(), 1):
        if i in drop:
            continue
        if i in comment_lines:
            line = line[:comment_lines[i]]
        line = re.sub(r'\s+', ' ', line).strip()
        if line:
            out.append(line)
    return out


def ratio(repo, ref):
    a = code_lines(repo)
    b = set(code_lines(ref))
    if not a:
        return 0.0, 0
    return sum(1 for x in a if x in b) / len(a), len(a)


if __name__ == '__main__':
    args = sys.argv[1:]
    for i in range(0, len(args), 2):
        r, n = ratio(args[i], args[i + 1])
        print(f'{100 * r:5.1f}%  ({n} lines)  {args[i]}  vs  {args[i + 1]}')
