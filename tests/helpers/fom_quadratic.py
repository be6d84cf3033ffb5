"""Fake evaluator command for HPO tests: prints a FoM line for a known quadratic."""
import argparse
import os

p = argparse.ArgumentParser()
p.add_argument("--x", type=float, default=0.5)
p.add_argument("--n", type=int, default=10)
p.add_argument("--opt", default="a")
a = p.parse_args()
if a.x > 0.97:                      # simulated crash: no FoM line
    raise SystemExit(3)
fom = (a.x - 0.3) ** 2 + (a.n - 5) ** 2 / 100.0 + (0.0 if a.opt == "b" else 0.5)
print("rank", os.environ.get("RANK", "-"), "visible", os.environ.get("HIP_VISIBLE_DEVICES", "-"))
print("FoM:", fom)
