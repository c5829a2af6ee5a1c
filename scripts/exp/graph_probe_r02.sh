# hipGraph update-capture repro matrix (scripts/exp/graph_update_repro.py), one process per variant
R=gpurun_out/probe3; mkdir -p $R
for args in "--variant sgd --env DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "--variant sgd --env TORCH_BLAS_PREFER_HIPBLASLT=0" "--variant sgd --env DEBUG_HIP_FORCE_GRAPH_QUEUES=1" "--variant sgd --env DEBUG_HIP_GRAPH_BATCH_SIZE=1" "--variant adam --churn" "--variant adam --churn --env DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "--variant sgd_zero"; do
  timeout -k 10 100 python -u scripts/exp/graph_update_repro.py $args >> $R/graph_update.jsonl 2>> $R/graph_update.err || echo "{\"fail\": \"$args\"}" >> $R/graph_update.jsonl
done
cat $R/graph_update.jsonl
timeout -k 10 100 python -u scripts/exp/timed_region_probe.py --reps 12 >> $R/timed.jsonl 2>>$R/timed.err && cat $R/timed.jsonl
