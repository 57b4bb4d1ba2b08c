#!/usr/bin/env python3
"""Runs GPU test functions in one process, in the given order, printing each
step (bisecting an order-dependent crash): repro_host_seq.py <module:function> ...
Fixtures disflow_mod / oracle are passed by name; parametrised tests take
their parameters as module:function[arg,arg]."""
import importlib
import inspect
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "optical-flow-using-dense-inverse-search_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import torch  # noqa: E402,F401

import disflow  # noqa: E402
import oracle_binding  # noqa: E402


def main():
    for spec in sys.argv[1:]:
        mod, fn = spec.split(":")
        args = []
        if "[" in fn:
            fn, a = fn[:-1].split("[")
            args = [int(x) for x in a.split(",") if x]
        f = getattr(importlib.import_module(mod), fn)
        kw = {}
        for name in inspect.signature(f).parameters:
            if name == "disflow_mod":
                kw[name] = disflow
            elif name == "oracle":
                kw[name] = oracle_binding
        params = [n for n in inspect.signature(f).parameters if n not in kw]
        kw.update(dict(zip(params, args)))
        print("run", spec, flush=True)
        f(**kw)
        print("  ok", flush=True)
    print("done", flush=True)


if __name__ == "__main__":
    main()
