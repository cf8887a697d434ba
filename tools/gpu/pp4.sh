set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
bash tools/gpu/pmc_conv.sh c4_l3c2 fwd 512,8,8,256,256,3,1,1 4
bash tools/gpu/pmc_conv.sh c6_l3c2 fwd 512,8,8,256,256,3,1,1 6
SDX_IGEMM_ABLATE=12 bash tools/gpu/pmc_conv.sh c6a12_l3c2 fwd 512,8,8,256,256,3,1,1 6
SDX_IGEMM_ABLATE=12 bash tools/gpu/pmc_conv.sh c4a12_l3c2 fwd 512,8,8,256,256,3,1,1 4
ls gpurun_out/pmc2 | head -50
bash tools/gpu/ablate_conv.sh fwd 512,8,8,256,256,3,1,1 "4 6" "0 2 10 14 6" > gpurun_out/pmc2/abl.txt 2>&1
cat gpurun_out/pmc2/abl.txt
