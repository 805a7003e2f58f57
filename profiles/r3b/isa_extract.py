"""Extract one kernel's ISA from the `make isa` listing: python isa_extract.py PATTERN OUT"""
import sys
txt = open("beam-radiance-estimate-pbrt_amd/csrc/build/isa/bre_gather.s").read().split("\n")
pat = sys.argv[1]
s = [i for i, l in enumerate(txt) if pat in l and not l.startswith((".", "\t", ";")) and ":" in l][0]
name = txt[s].split(":")[0]
e = [i for i in range(s, len(txt)) if txt[i].strip().startswith("s_endpgm")][0]
open(sys.argv[2], "w").write("\n".join(txt[s:e + 1]))
print(name, e - s)
