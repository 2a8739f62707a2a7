"""Extract the surf_usage known answers into tests/golden/surf_usage.json (run once where /root/reference exists):
    python tests/golden/make_surf_usage.py
It reads ONLY data: the expected-output lines of teshsuite/surf/surf_usage/surf_usage.tesh and
surf_usage2/surf_usage2.tesh (the surf_test/INFO lines: clock and message), and the three profile files of
examples/platforms/two_hosts_profiles.xml (examples/platforms/profiles/trace_A.txt, trace_A_failure.txt,
trace_B.txt: dated values).  tests/surf_scenario.py restates the scenario and replays it against them."""
import json
import os

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


def tesh_lines(path):
    res = []
    with open(path) as f:
        for line in f:
            if line.startswith("> [") and "[surf_test/INFO]" in line:
                res.append([line[3:line.index("]")], line.split("[surf_test/INFO] ", 1)[1].rstrip("\n")])
    return res


def main():
    out = {"expected": {}, "profiles": {}}
    for name in ("surf_usage", "surf_usage2"):
        out["expected"][name] = tesh_lines(os.path.join(REF, "teshsuite", "surf", name, name + ".tesh"))
    for p in ("trace_A.txt", "trace_A_failure.txt", "trace_B.txt"):
        with open(os.path.join(REF, "examples", "platforms", "profiles", p)) as f:
            out["profiles"][p] = f.read()
    with open(os.path.join(HERE, "surf_usage.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", os.path.join(HERE, "surf_usage.json"))


if __name__ == "__main__":
    main()
