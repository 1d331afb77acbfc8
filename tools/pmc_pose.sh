set -e -o pipefail
R=$(pwd); O=$R/gpurun_out/pmcpose; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_VALU --kernel-trace -d $O/a -o run --output-format csv -- python3 $R/tools/pose_bench.py --batch 256 --steps 2 --warmup 1 --no-cpu > $O/a.json 2> $O/a.err
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAVES GRBM_GUI_ACTIVE SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 --kernel-trace -d $O/b -o run --output-format csv -- python3 $R/tools/pose_bench.py --batch 256 --steps 2 --warmup 1 --no-cpu > $O/b.json 2> $O/b.err
cd $R; python tools/pmc_table.py gpurun_out/pmcpose
