set -o pipefail
O=gpurun_out/r05g; mkdir -p $O
for v in default abx/libmlamg_hot0.so abx/libmlamg_hot512.so abx/libmlamg_hot2048.so abx/libmlamg_hot4096.so; do
  if [ "$v" = default ]; then L=ml-amg_amd/mlamg/libmlamg_hip.so; else L=tools/$v; fi
  MLAMG_LIB=$L timeout -k 10 300 python -u tools/vc_ab.py --tag $L >> $O/vc_ab.jsonl 2>> $O/vc_ab.err || exit 1
done
