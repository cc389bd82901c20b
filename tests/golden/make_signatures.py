#!/usr/bin/env python3
"""Write tests/golden/ref_signatures.json: the parameter lists (names and default
expressions, as source text) of every method of the reference's plugin and solver
classes on the north-star path, read with `ast` from the reference's sources (no
import, nothing executed).  Test infrastructure: the data is compared with this
build's classes by tests/test_signatures.py, here and without /root/reference.

Usage:  python tests/golden/make_signatures.py
"""
import ast
import json
import os

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "ref_signatures.json")
FILES = {
    "TrajoptMPCReference.py": ["TrajoptMPCReference"],
    "TrajoptPlant.py": ["TrajoptPlant", "URDFPlant"],
    "TrajoptCost.py": ["TrajoptCost", "QuadraticCost", "UrdfCost"],
    "TrajoptConstraint.py": ["BoxConstraint", "TrajoptConstraint"],
    "GBD-PCG-Python/PCG.py": ["PCG"],
}


def main():
    out = {}
    for rel, classes in FILES.items():
        tree = ast.parse(open(os.path.join(REF, rel)).read())
        for cls in tree.body:
            if not isinstance(cls, ast.ClassDef) or cls.name not in classes:
                continue
            for fn in cls.body:
                if not isinstance(fn, ast.FunctionDef):
                    continue
                a = fn.args
                names = [x.arg for x in a.args]
                defs = [None] * (len(names) - len(a.defaults)) + [ast.unparse(d) for d in a.defaults]
                out[f"{cls.name}.{fn.name}"] = {"source": f"{rel}:{fn.lineno}",
                                                "params": [[n, d] for n, d in zip(names, defs)],
                                                "varargs": a.vararg is not None, "kwargs": a.kwarg is not None}
    with open(OUT, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(f"{len(out)} signatures -> {OUT}")


if __name__ == "__main__":
    main()
