# PMC counters of the 3x3 64 / 128-channel conv kernels (layer1.1 / layer2.1 conv2 shapes); one pass each
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/c3_pmc; mkdir -p $OUT
export ONLY=layer1.1,layer2.1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_INSTS_SALU --output-format csv -d $OUT/p1 -o run -- python tools/probes/resnet_layers.py --reps 3 > $OUT/p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM --output-format csv -d $OUT/p2 -o run -- python tools/probes/resnet_layers.py --reps 3 > $OUT/p2.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES --output-format csv -d $OUT/p3 -o run -- python tools/probes/resnet_layers.py --reps 3 > $OUT/p3.log 2>&1 || exit 1
echo done
