import sys, importlib, numpy as np, torch
sys.path.insert(0,'tests'); sys.path.insert(0,'.')
from oracle import dataset_ref as D
from test_dataset_gpu import _frames
pkg=importlib.import_module('image-segmentation-project_amd')
f=_frames(1,3,96,160)
got=pkg.preprocess(f, img_size=(160,96)).cpu().numpy()[:,0]
for i in range(3):
    want=D.normalize_microscopy_image(f[i]).astype(np.float32)
    d=np.argwhere(got[i]!=want)
    print(i, len(d), d[:10].tolist())
    c=D.clahe_u8(np.clip(f[i],*np.percentile(f[i],[2,98])).astype(np.uint8))
    rng=c.max()-c.min()
    for (y,x) in d[:5]:
        print('  ', y, x, 'got', got[i,y,x]*rng, 'want', want[y,x]*rng)
