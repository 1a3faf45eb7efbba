"""Count instructions of one kernel in a hipcc --save-temps .s file:
python tools/isa_count.py file.s k_render_fwd  -> total VALU / SALU / packed / ds / vmem."""
import re
import sys

path, name = sys.argv[1], sys.argv[2]
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*" + name + r"\S*:", l))
body = []
for l in lines[start + 1:]:
    if "s_endpgm" in l:
        break
    body.append(l.strip())
ins = [l.split()[0] for l in body if l and not l.startswith((";", ".", "_"))]
cnt = lambda p: sum(1 for i in ins if i.startswith(p))
print(f"{name}: total {len(ins)}  v_ {cnt('v_')}  v_pk_ {cnt('v_pk_')}  s_ {cnt('s_')}  ds_ {cnt('ds_')}  "
      f"global_ {cnt('global_')}  exec-branches {cnt('s_cbranch')}")
