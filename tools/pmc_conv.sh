cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
S=512,8,8,256,256,3,1,1
timeout -k 10 120 python tools/conv_one.py --mode fwd --shape $S > gpurun_out/pmc_t.txt 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY --output-format csv -d gpurun_out/pmc1 -o run -- python tools/conv_one.py --mode fwd --shape $S --iters 5 > gpurun_out/pmc1.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d gpurun_out/pmc2 -o run -- python tools/conv_one.py --mode fwd --shape $S --iters 5 > gpurun_out/pmc2.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE --output-format csv -d gpurun_out/pmc3 -o run -- python tools/conv_one.py --mode fwd --shape $S --iters 5 > gpurun_out/pmc3.log 2>&1 || exit 1
