cd $GRAFT_REPO_ROOT && export PYTHONPATH=$PWD && mkdir -p gpurun_out/r3g &&
timeout -k 10 300 python tools/gemm_bench.py --variants 8,11 --dbg 0,1,2,4 --iters 20 --only bert_qkv_fwd,bert_ffn1_fwd,bert_ffn2_fwd,bert_ffn2_dgrad,sq8192 --out gpurun_out/r3g/gemm_stagger.jsonl > gpurun_out/r3g/gemm_bench.log 2>&1
