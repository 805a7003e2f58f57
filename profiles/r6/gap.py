#!/usr/bin/env python3
"""Pipeline gaps from a rocprofv3 kernel trace of the pipelined C2 bench: for every consecutive pair of
k_gather_tile dispatches, the gap between one's end and the next one's start, and where the passes of
the next iteration ran (the photon kernel's start / end relative to the running gather).
usage: gap.py run_kernel_trace.csv [label]"""
import csv
import statistics as stt
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
lab = sys.argv[2] if len(sys.argv) > 2 else ""
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
G = [r for r in rows if "k_gather_tile" in r["Kernel_Name"]]
P = [r for r in rows if "k_photons<2>" in r["Kernel_Name"] or "k_photons<0>" in r["Kernel_Name"]]
gaps, pdur, plate, chain = [], [], [], []
for i in range(len(G) - 1):
    gs, ge = int(G[i]["Start_Timestamp"]), int(G[i]["End_Timestamp"])
    ns = int(G[i + 1]["Start_Timestamp"])
    gaps.append((ns - ge) / 1e6)
    ph = [p for p in P if gs <= int(p["Start_Timestamp"]) < ge]
    if ph:
        p = ph[0]
        pdur.append((int(p["End_Timestamp"]) - int(p["Start_Timestamp"])) / 1e6)
        plate.append((int(p["End_Timestamp"]) - ge) / 1e6)  # > 0: the photon pass ended after the gather
        chain.append((ns - int(p["End_Timestamp"])) / 1e6)
def med(x):
    return round(stt.median(x), 3) if x else None
print(f"{lab} gathers {len(G)} gap_ms mean {round(stt.mean(gaps), 3) if gaps else None} median {med(gaps)} "
      f"| photon kernel during a gather: n {len(pdur)} dur median {med(pdur)} end-after-gather median {med(plate)} "
      f"| photon end -> next gather start median {med(chain)}")
