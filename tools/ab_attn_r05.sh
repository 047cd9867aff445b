# GPU box: spatial / temporal attention timing, env variants interleaved (tools/attn_bench.py)
#   bash tools/ab_attn_r05.sh "<name>|<env>" ["<name>|<env>" ...]
for r in 1 2; do
  for v in "$@"; do
    n=${v%%|*}; e=${v#*|}
    echo "== $n $r"
    env $e timeout -k 10 120 python -u tools/attn_bench.py || exit 1
  done
done
