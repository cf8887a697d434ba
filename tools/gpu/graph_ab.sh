set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/gab
mkdir -p $O
for spec in "eager:--graph 0" "g:--graph 1" "g_nopc:--graph 1|DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "g_q4:--graph 1|DEBUG_HIP_FORCE_GRAPH_QUEUES=4" "g_q4nopc:--graph 1|DEBUG_HIP_FORCE_GRAPH_QUEUES=4 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0"; do
  tag=${spec%%:*}; rest=${spec#*:}; args=${rest%%|*}; envs=""; [[ "$rest" == *"|"* ]] && envs=${rest#*|}
  for b in 256 128; do
    env $envs timeout -k 10 150 python bench.py --steps 30 --warmup 10 --per_gpu_batch $b $args > $O/${tag}_$b.txt 2>&1 || { echo "$tag $b failed"; tail -3 $O/${tag}_$b.txt; continue; }
    echo "$tag b$b $(grep -o '"ms_per_step": [0-9.]*' $O/${tag}_$b.txt) | $(grep -o 'host issue time (idle queue) [0-9.]*' $O/${tag}_$b.txt)"
  done
done
