"""``CViT-main/helpers/loader.py`` import path (cvit_prediction.py:19 puts
``helpers/`` on sys.path).  What the inference path shares with it are the
ImageNet normalisation constants (loader.py:9-10 = cvit_prediction.py:41-42),
which the gfx950 path fuses into conv1 (fac_fake_amd/csrc/stem224.hip).  The
training loaders (ImageFolder + albumentations, loader.py:17-60) are outside
the inference path."""
mean = [0.485, 0.456, 0.406]
std = [0.229, 0.224, 0.225]
