"""Extract the dragonfly known answers into tests/golden/dragonfly_coords.json (run once where /root/reference
exists):
    python tests/golden/make_dragonfly_coords.py
It reads ONLY data:
  * the expected-output lines of examples/s4u/routing-get-clusters/s4u-routing-get-clusters.tesh for its
    cluster_dragonfly.xml run: the cluster's host names (one line each) and the `rank: (group, chassis, blade, node)`
    lines DragonflyZone::rankId_to_coords produces (DragonflyZone.cpp:26-35);
  * the <cluster> element of examples/platforms/cluster_dragonfly.xml: its topo_parameters and radical.
tests/test_platforms.py requires the product's (lmm_platform_dragonfly_coords) and the oracle's (oracle/platforms.py)
coordinates and host count to be these."""
import json
import os
import re

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
TESH = os.path.join(REF, "examples/s4u/routing-get-clusters/s4u-routing-get-clusters.tesh")
XML = os.path.join(REF, "examples/platforms/cluster_dragonfly.xml")


def main():
    hosts, coords, run, section = [], [], False, None
    with open(TESH) as f:
        for line in f:
            if line.startswith("$ "):
                run = "cluster_dragonfly.xml" in line
                continue
            if not run or not line.startswith("> ["):
                continue
            msg = re.match(r"> \[\s*[0-9.]+\] \([^)]*\) (.*)$", line.rstrip("\n")).group(1)
            if msg.endswith("dragonfly topology:"):
                section = "coords"
            elif not msg.startswith("   "):
                section = "hosts"
            elif section == "hosts":
                hosts.append(msg.strip())
            else:
                m = re.match(r"\s*(\d+): \((\d+), (\d+), (\d+), (\d+)\)$", msg)
                coords.append([int(m.group(i)) for i in range(1, 6)])
    xml = open(XML).read()
    topo = re.search(r'topology="DRAGONFLY" topo_parameters="([^"]+)"', xml).group(1)
    radical = re.search(r'radical="([^"]+)"', xml).group(1)
    out = {"source": "examples/s4u/routing-get-clusters/s4u-routing-get-clusters.tesh (cluster_dragonfly.xml run), "
                     "examples/platforms/cluster_dragonfly.xml",
           "topo_parameters": topo, "radical": radical, "hosts": hosts,
           "coords": coords}
    with open(os.path.join(HERE, "dragonfly_coords.json"), "w") as f:
        json.dump(out, f, indent=0)
    print(f"{len(hosts)} hosts, {len(coords)} coordinate lines, topo {topo}")


if __name__ == "__main__":
    main()
