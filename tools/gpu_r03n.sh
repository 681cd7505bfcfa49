set -eo pipefail
mkdir -p gpurun_out/r03n
for spec in "20 10" "16 8"; do set -- $spec
timeout -k 10 200 python -u tools/dec_select.py --k $1 --m $2 --blocks 524288 --rounds 7 --only "wpc,vector" > gpurun_out/r03n/single_$1.log 2>&1
tail -1 gpurun_out/r03n/single_$1.log; done
