"""AST-extract the reference's training classes (build container only).

Coop-MH-PPO-scalable.py cannot be imported (input() at :1011, train(1000) at
:1062): exec only its Import/ClassDef/FunctionDef nodes above line 1003,
dropping matplotlib, then inject the globals the classes read (`env`,
`nb_lines`).  Notebook drivers: same, from the code cell
holding `class Algo_PPO`.
"""
import ast
import json

import refharness  # noqa: F401  (sets up sys.path / gym stub)

SCRIPT = "/root/reference/Coop-MH-PPO-scalable.py"
NOTEBOOKS = {"coop": ("/root/reference/Coop-MH-PPO.ipynb", 0), "naif": ("/root/reference/MH-PPO.ipynb", 1)}


def _exec_nodes(src, max_line=None, **globs):
    tree = ast.parse(src)
    keep = []
    for node in tree.body:
        if max_line is not None and node.lineno >= max_line:
            continue
        if isinstance(node, (ast.Import, ast.ImportFrom)):
            names = [a.name for a in node.names]
            mod = getattr(node, "module", None) or ""
            if any("matplotlib" in n for n in names) or "matplotlib" in mod:
                continue
            keep.append(node)
        elif isinstance(node, (ast.ClassDef, ast.FunctionDef)):
            keep.append(node)
    ns = dict(globs)
    exec(compile(ast.Module(body=keep, type_ignores=[]), "<reference>", "exec"), ns)
    return ns


def scalable_classes(**globs):
    return _exec_nodes(open(SCRIPT).read().replace("\r", ""), max_line=1003, **globs)


def notebook_classes(which, **globs):
    path, cell = NOTEBOOKS[which]
    nb = json.load(open(path))
    src = "".join(nb["cells"][cell]["source"]).replace("\r", "")
    return _exec_nodes(src, **globs)
