"""Extract the s4u-app-pingpong known answers into tests/golden/pingpong.json (run once where /root/reference
exists):
    python tests/golden/make_pingpong.py
It reads ONLY data:
  * the expected-output lines of examples/s4u/app-pingpong/s4u-app-pingpong.tesh for its three LMM runs —
    default (LV08, Lazy), `--cfg=network/optim:Full` (LV08, Full) and `--cfg=network/model:CM02` (CM02,
    Lazy) — as (clock, actor@host or "maestro", message), the "Configuration change" lines dropped; the fourth
    run (network/model:Constant) has no LMM system and is not taken;
  * the one link of the Tremblay -> Jupiter route of examples/platforms/small_platform.xml (the <route> between
    them and that <link>'s bandwidth / latency attributes, converted to B/s and s).
tests/pingpong_scenario.py restates the scenario and replays it against them."""
import json
import os
import re

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
RUNS = [("lv08_lazy", None), ("lv08_full", "network/optim:Full"), ("cm02_lazy", "network/model:CM02")]


def tesh_runs(path):
    """The `$ ...` commands of the tesh file and their `> ` lines."""
    runs, cur = [], None
    with open(path) as f:
        for line in f:
            if line.startswith("$ "):
                cur = {"cmd": line[2:].strip(), "lines": []}
                runs.append(cur)
            elif line.startswith("> [") and cur is not None:
                m = re.match(r"> \[\s*([0-9.]+)\] \(([^)]*)\) (.*)$", line.rstrip("\n"))
                if m and "Configuration change" not in m.group(3):
                    who = m.group(2).split(":", 1)[1]  # "1:pinger@Tremblay" -> "pinger@Tremblay"
                    runs[-1]["lines"].append([m.group(1), who, m.group(3)])
    return runs


def unit(v, units):
    m = re.match(r"([0-9.eE+-]+)([A-Za-z]*)$", v)
    return float(m.group(1)) * units[m.group(2)]


def main():
    runs = tesh_runs(os.path.join(REF, "examples", "s4u", "app-pingpong", "s4u-app-pingpong.tesh"))
    out = {"expected": {}}
    for name, cfg in RUNS:
        sel = [r for r in runs if "small_platform.xml" in r["cmd"] and
               (cfg is None and "--cfg" not in r["cmd"] or cfg is not None and cfg in r["cmd"])]
        assert len(sel) == 1, (name, [r["cmd"] for r in sel])
        out["expected"][name] = sel[0]["lines"]
    with open(os.path.join(REF, "examples", "platforms", "small_platform.xml")) as f:
        xml = f.read()
    route = re.search(r'<route src="Tremblay" dst="Jupiter">(.*?)</route>', xml, re.S).group(1)
    ids = re.findall(r'<link_ctn id="([^"]+)"/>', route)
    links = []
    for lid in ids:
        m = re.search(r'<link id="%s" bandwidth="([^"]+)" latency="([^"]+)"' % re.escape(lid), xml)
        links.append({"id": lid, "bw": unit(m.group(1), {"MBps": 1e6, "kBps": 1e3, "Bps": 1.0, "GBps": 1e9}),
                      "lat": unit(m.group(2), {"ms": 1e-3, "us": 1e-6, "s": 1.0, "ns": 1e-9})})
    out["route_tremblay_jupiter"] = links
    with open(os.path.join(HERE, "pingpong.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", os.path.join(HERE, "pingpong.json"))


if __name__ == "__main__":
    main()
