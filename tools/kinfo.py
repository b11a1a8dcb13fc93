"""Register / scratch / LDS use of every kernel in a device assembly file (hipcc -S output)."""
import re
import sys

txt = open(sys.argv[1]).read()
pat = sys.argv[2] if len(sys.argv) > 2 else ""
for blk in txt.split("- .agpr_count:")[1:]:
    def g(k):
        m = re.search(r"\." + k + r":\s+(\S+)", blk)
        return m.group(1) if m else "?"
    name = g("name")
    if pat in name:
        print(f"{name:70s} vgpr {g('vgpr_count'):>4} spill {g('vgpr_spill_count'):>4} scratch {g('private_segment_fixed_size'):>4} "
              f"lds {g('group_segment_fixed_size'):>6} sgpr {g('sgpr_count'):>4}")
