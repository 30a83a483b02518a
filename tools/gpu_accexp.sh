set -e
cd ${GRAFT_REPO_ROOT}
mkdir -p gpurun_out/$1
for spec in "64,64,64,128 --stride 2" "64,128,32,256 --stride 2" "64,256,16,512 --stride 2" "64,64,64,64" "64,128,32,128" "64,256,16,256" "64,512,8,512"; do
  for acc in "" "--acc"; do
    timeout -k 10 60 python tools/conv_exp.py --shape $spec --phase dgrad $acc >> gpurun_out/$1/acc.jsonl
  done
done
cat gpurun_out/$1/acc.jsonl
