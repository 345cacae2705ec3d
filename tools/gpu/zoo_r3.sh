#!/bin/bash
# native-only whole-zoo pass at bs256 (round 3): every family + the odd-width grouped nets that
# now run their group pad / slice / channel shuffle as native remaps
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/zoo3
for m in LeNet VGG16 ResNet18 ResNet50 PreActResNet18 GoogLeNet DenseNet121 densenet_cifar ResNeXt29_2x64d \
         ResNeXt29_32x4d MobileNet MobileNetV2 DPN26 ShuffleNetG2 ShuffleNetG3 ShuffleNetV2_1 SENet18 \
         EfficientNetB0 RegNetX_200MF RegNetY_400MF SimpleDLA DLA PNASNetA PNASNetB; do
  timeout -k 10 150 python bench.py --model $m --batch 256 --steps 10 --warmup 3 > gpurun_out/zoo3/$m.json 2> gpurun_out/zoo3/$m.err
  rc=$?
  if [ $rc -ne 0 ]; then echo "$m FAILED rc=$rc"; tail -3 gpurun_out/zoo3/$m.err; [ $rc -ge 124 ] && exit 1; continue; fi
  python3 -c "import json; d=json.loads(open('gpurun_out/zoo3/$m.json').read().strip().splitlines()[-1]); print('$m', d['ms_per_step'], d['value'])"
done
