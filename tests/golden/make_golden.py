"""Extract golden vectors from the reference's own tesh files into small JSON fixtures.

Run once in the build container (where /root/reference exists):
    python tests/golden/make_golden.py
It reads ONLY the expected-output text of
    teshsuite/surf/maxmin_bench/maxmin_bench_{small,medium}.tesh
    teshsuite/surf/maxmin_bench/maxmin_bench_large.tesh
and writes tests/golden/maxmin_bench_{small,medium,large}.json.  The fixtures are data
(inputs implied by the seeded generator + expected outputs), not reference source.

What the tesh output pins (maxmin_bench in `test` mode runs System::lmm_solve with
surf/maxmin at DEBUG, maxmin.cpp:541-542 and System::print(), maxmin.cpp:441-485):
  * "Starting i: (x)" / "Starting to solve(y)"  -> RNG stream checks      (maxmin_bench.cpp:178,80)
  * "Constraint 'r' usage: U remaining: R concurrency: a<=b<=c"  -> init state (maxmin.cpp:541)
  * "MAX-MIN ( 'r'(p) ... )"                    -> variable_set order + penalties
  * "\t(w.'r'(x) + ... + 0) <= B ('r')"         -> per-constraint element list (enabled then
                                                   disabled, list order), weights, bound
  * "'r'(p) : x"                                -> solved variable values
  * "Setting var (r) value to x"                -> the value each variable was fixed at
All numbers are printed with %f (6 decimals).  Ranks are global static counters
(maxmin.cpp:22-23): run k of a class with V variables owns variable ranks k*V+1 .. k*V+V.
"""
import json
import os
import re
import sys

REF = "/root/reference/teshsuite/surf/maxmin_bench"
HERE = os.path.dirname(os.path.abspath(__file__))

RX_START = re.compile(r"Starting (\d+): \((\d+)\)")
RX_SOLVE = re.compile(r"Starting to solve\((\d+)\)")
RX_INIT = re.compile(r"Constraint '(\d+)' usage: ([0-9.]+) remaining: ([0-9.]+) concurrency: (-?\d+)<=(-?\d+)<=(-?\d+)")
RX_OBJ = re.compile(r"MAX-MIN \( (.*)\)$")
RX_OBJ_TERM = re.compile(r"'(\d+)'\(([0-9.]+)\)")
RX_EQ = re.compile(r"\t(max)?\((.*)0\) <= ([0-9.]+) \('(\d+)'\)( \[MAX-Constraint\])?$")
RX_TERM = re.compile(r"([0-9.]+)\.'(\d+)'\(([0-9.]+)\)")
RX_VAR = re.compile(r"\] '(\d+)'\(([0-9.]+)\) : ([0-9.]+)$")
RX_SET = re.compile(r"Setting var \((\d+)\) value to ([0-9.]+)")

CLASSES = {"small": (10, 10), "medium": (100, 100)}


def parse(name, nruns):
    C, V = CLASSES[name]
    runs = [dict(run=k, seed=k + 1, init={}, objective=[], constraints={}, values={}, set_values={},
                 check_start=None, check_solve=None) for k in range(nruns)]
    starts = []
    solves = []
    with open(os.path.join(REF, f"maxmin_bench_{name}.tesh")) as f:
        for line in f:
            line = line.rstrip("\n")
            if not line.startswith(">"):
                continue
            m = RX_START.search(line)
            if m:
                starts.append((int(m.group(1)), int(m.group(2))))
                continue
            m = RX_SOLVE.search(line)
            if m:
                solves.append(int(m.group(1)))
                continue
            m = RX_INIT.search(line)
            if m:
                rank = int(m.group(1))
                run = (rank - 1) // C
                runs[run]["init"][rank - run * C] = [float(m.group(2)), float(m.group(3)),
                                                     int(m.group(4)), int(m.group(5)), int(m.group(6))]
                continue
            m = RX_OBJ.search(line)
            if m:
                terms = [(int(a), float(b)) for a, b in RX_OBJ_TERM.findall(m.group(1))]
                run = (terms[0][0] - 1) // V
                runs[run]["objective"] = [[r - run * V, p] for r, p in terms]
                continue
            m = RX_EQ.search(line)
            if m:
                rank = int(m.group(4))
                run = (rank - 1) // C
                terms = [[int(r) - run * V, float(w)] for w, r, _x in RX_TERM.findall(m.group(2))]
                runs[run]["constraints"][rank - run * C] = dict(bound=float(m.group(3)),
                                                                 fatpipe=bool(m.group(1)), elems=terms)
                continue
            m = RX_VAR.search(line)
            if m:
                rank = int(m.group(1))
                run = (rank - 1) // V
                runs[run]["values"][rank - run * V] = [float(m.group(2)), float(m.group(3))]
                continue
            m = RX_SET.search(line)
            if m:
                rank = int(m.group(1))
                run = (rank - 1) // V
                runs[run]["set_values"][rank - run * V] = float(m.group(2))
    # Starting i / Starting to solve lines are emitted in pairs, in run order
    for (i, x), y in zip(starts, solves):
        runs[i]["check_start"] = x
        runs[i]["check_solve"] = y
    for r in runs:
        # distinct fixing levels = outer rounds of the reference's progressive filling
        r["distinct_set_levels"] = len(set(r["set_values"].values()))
        for key in ("init", "constraints", "values", "set_values"):
            r[key] = {str(k): v for k, v in sorted(r[key].items())}
    return dict(source=f"teshsuite/surf/maxmin_bench/maxmin_bench_{name}.tesh", klass=name,
                nb_cnst=C, nb_var=V, runs=runs)


def parse_large():
    out = {}
    with open(os.path.join(REF, "maxmin_bench_large.tesh")) as f:
        for line in f:
            m = RX_START.search(line)
            if m:
                out["check_start"] = int(m.group(2))
            m = RX_SOLVE.search(line)
            if m:
                out["check_solve"] = int(m.group(1))
    return dict(source="teshsuite/surf/maxmin_bench/maxmin_bench_large.tesh", klass="big", run=0, **out)


def main():
    if not os.path.isdir(REF):
        sys.exit("reference not present; fixtures are already committed")
    for name, n in (("small", 10), ("medium", 5)):
        d = parse(name, n)
        with open(os.path.join(HERE, f"maxmin_bench_{name}.json"), "w") as f:
            json.dump(d, f, separators=(",", ":"))
    with open(os.path.join(HERE, "maxmin_bench_large.json"), "w") as f:
        json.dump(parse_large(), f, indent=1)


if __name__ == "__main__":
    main()
