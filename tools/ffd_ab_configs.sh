set -e
for k in 1 2; do
for lib in libgpusched.so libgpusched_reg.so; do
  for c in --c1 --c2 ""; do
    ms=$(GPUSCHED_LIB=$lib timeout -k 10 120 python3 tools/ffd_diag.py $c | python3 -c 'import json,sys; d=json.load(sys.stdin); print(round(d["ffd_ms"],2), d["claims"])')
    echo "$lib $c $ms"
  done
done
done
