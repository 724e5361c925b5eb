set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/fapmc
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU --kernel-trace --output-format csv -d $R/gpurun_out/fapmc/a -o run -- python3 $R/scripts/fa_only.py 1024 > $R/gpurun_out/fapmc/a.log 2>&1 || { tail $R/gpurun_out/fapmc/a.log; exit 1; }
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --kernel-trace --output-format csv -d $R/gpurun_out/fapmc/b -o run -- python3 $R/scripts/fa_only.py 1024 > $R/gpurun_out/fapmc/b.log 2>&1 || { tail $R/gpurun_out/fapmc/b.log; exit 1; }
timeout -k 10 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT --kernel-trace --output-format csv -d $R/gpurun_out/fapmc/c -o run -- python3 $R/scripts/fa_only.py 1024 > $R/gpurun_out/fapmc/c.log 2>&1 || { tail $R/gpurun_out/fapmc/c.log; exit 1; }
echo done
