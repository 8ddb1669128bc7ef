# hipBLASLt solution tuning (PyTorch TunableOp) for BERT's remaining library GEMMs, then the
# bench with and without the tuned table, same box
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --model bert_base --steps 3 --warmup 2 --gemm-tuning tune \
  --gemm-tuning-out gpurun_out/tunableop_bert_base.csv > gpurun_out/r4_tune_bert.json 2> gpurun_out/r4_tune_bert.err || exit 1
cp gpurun_out/tunableop_bert_base.csv distributedtensorflow_amd/tuning/tunableop_bert_base.csv || exit 1
timeout -k 10 200 python bench.py --model bert_base > gpurun_out/r4_bench_bert_tuned.json 2> gpurun_out/r4_bench_bert_tuned.err && \
timeout -k 10 200 python bench.py --model bert_base --gemm-tuning off > gpurun_out/r4_bench_bert_untuned.json 2> gpurun_out/r4_bench_bert_untuned.err && \
timeout -k 10 200 python bench.py --model bert_base > gpurun_out/r4_bench_bert_tuned2.json 2> gpurun_out/r4_bench_bert_tuned2.err
