"""get_transform (reference: visreps/dataloaders/obj_cls.py:27-45) on the device against
Pillow + numpy. CPU: the numpy restatement of Pillow's resample (oracle/transform_oracle.py)
is pinned to Pillow's own Image.resize on seeded images. GPU: vr_transform_u8 equals
torchvision's result on PIL images bit for bit (Pillow resize + center crop + fp32
/255, -mean, /std, each op rounded once)."""
import numpy as np
import pytest

from oracle import transform_oracle as T

SIZES = [(425, 425), (300, 500), (512, 256), (256, 256), (240, 320), (1000, 700), (257, 300), (64, 90)]


def _img(h, w, seed):
    rs = np.random.RandomState(seed)
    # smooth field + noise, so both flat and sharp regions are exercised
    base = rs.rand(h // 8 + 2, w // 8 + 2, 3)
    yy = np.linspace(0, base.shape[0] - 1.001, h)
    xx = np.linspace(0, base.shape[1] - 1.001, w)
    smooth = base[yy.astype(int)][:, xx.astype(int)]
    return np.clip(smooth * 255 + rs.randn(h, w, 3) * 20, 0, 255).astype(np.uint8)


def _pil_ref(img, resize, crop, mean, std, kind="bilinear"):
    from PIL import Image

    H, W, _ = img.shape
    nh, nw = T.resize_size(H, W, resize)
    f = Image.BICUBIC if kind == "bicubic" else Image.BILINEAR
    r = np.asarray(Image.fromarray(img, "RGB").resize((nw, nh), f))
    top, left = int(round((nh - crop) / 2.0)), int(round((nw - crop) / 2.0))
    c = r[top:top + crop, left:left + crop]
    x = np.transpose(c, (2, 0, 1)).astype(np.float32) / np.float32(255)
    return ((x - np.asarray(mean, np.float32)[:, None, None]) / np.asarray(std, np.float32)[:, None, None])


@pytest.mark.parametrize("h,w", SIZES[:6])
def test_oracle_resample_matches_pillow(h, w):
    from PIL import Image

    img = _img(h, w, h * 7 + w)
    for nw, nh in [T.resize_size(h, w, 256)[::-1], (w // 3 + 1, h // 2 + 5), (w + 37, h + 11)]:
        ref = np.asarray(Image.fromarray(img, "RGB").resize((nw, nh), Image.BILINEAR))
        assert np.array_equal(T.resample(img, nw, nh), ref)


@pytest.mark.parametrize("h,w", [(425, 425), (300, 500), (240, 320), (64, 90)])
def test_oracle_bicubic_resample_matches_pillow(h, w):
    from PIL import Image

    img = _img(h, w, h + 3 * w)
    for nw, nh in [T.resize_size(h, w, 224)[::-1], (w + 19, h + 7)]:
        ref = np.asarray(Image.fromarray(img, "RGB").resize((nw, nh), Image.BICUBIC))
        assert np.array_equal(T.resample(img, nw, nh, "bicubic"), ref)


def test_oracle_transform_matches_pil_pipeline():
    from visreps_amd.dataloaders.obj_cls import DS_MEAN, DS_STD

    img = _img(300, 500, 1)
    got = T.transform(img, 256, 224, DS_MEAN["imgnet"], DS_STD["imgnet"])
    assert np.array_equal(got, _pil_ref(img, 256, 224, DS_MEAN["imgnet"], DS_STD["imgnet"]))


def test_get_transform_refuses_augmentation():
    from visreps_amd.dataloaders.obj_cls import get_transform

    with pytest.raises(NotImplementedError):
        get_transform(data_augment=True)
    t = get_transform("tiny-imagenet")
    assert (t.resize, t.crop) == (64, 64)


@pytest.mark.gpu
@pytest.mark.parametrize("h,w", SIZES)
def test_transform_bit_exact_vs_pillow(dev, h, w):
    from visreps_amd.dataloaders.obj_cls import DS_MEAN, DS_STD, get_transform

    t = get_transform("imgnet")
    imgs = [_img(h, w, s) for s in range(3)]
    got = t.batch(imgs).cpu().numpy()
    assert got.shape == (3, 3, 224, 224)
    for i, im in enumerate(imgs):
        ref = _pil_ref(im, 256, 224, DS_MEAN["imgnet"], DS_STD["imgnet"])
        assert np.array_equal(got[i], ref), np.abs(got[i] - ref).max()


@pytest.mark.gpu
def test_transform_mixed_sizes_pil_inputs_and_tiny(dev):
    from PIL import Image
    from visreps_amd.dataloaders.obj_cls import DS_MEAN, DS_STD, get_transform

    imgs = [_img(300, 500, 3), _img(425, 425, 4), _img(300, 500, 5)]
    pil = [Image.fromarray(imgs[0], "RGB"), Image.fromarray(imgs[1], "RGB").convert("RGBA"), imgs[2]]
    t = get_transform("imgnet")
    got = t.batch(pil).cpu().numpy()
    for i, im in enumerate(imgs):
        assert np.array_equal(got[i], _pil_ref(im, 256, 224, DS_MEAN["imgnet"], DS_STD["imgnet"]))
    tiny = get_transform("tiny-imagenet")
    g = tiny(imgs[1]).cpu().numpy()
    assert np.array_equal(g, _pil_ref(imgs[1], 64, 64, DS_MEAN["tiny-imagenet"], DS_STD["tiny-imagenet"]))


@pytest.mark.gpu
def test_image_loader_order_and_paths(dev, tmp_path):
    from PIL import Image
    from visreps_amd.dataloaders.neural import _make_loader
    from visreps_amd.dataloaders.obj_cls import DS_MEAN, DS_STD, get_transform

    stim = {}
    for k in ["b", "a", "10", "2"]:
        p = tmp_path / f"{k}.png"
        Image.fromarray(_img(260, 300, len(k) + ord(k[0])), "RGB").save(p)
        stim[k] = str(p)
    batches = list(_make_loader(stim, get_transform("imgnet"), 3, 0))
    keys = [k for _, ks in batches for k in ks]
    assert keys == sorted(stim)
    first = batches[0][0].cpu().numpy()
    ref = _pil_ref(np.asarray(Image.open(stim["10"]).convert("RGB")), 256, 224, DS_MEAN["imgnet"], DS_STD["imgnet"])
    assert np.array_equal(first[0], ref)


@pytest.mark.gpu
@pytest.mark.parametrize("h,w", [(425, 425), (300, 500), (512, 256), (1000, 700), (64, 90)])
def test_clip_and_dino_transforms_bit_exact_vs_pillow_bicubic(dev, h, w):
    from visreps_amd.dataloaders.obj_cls import DS_MEAN, DS_STD, clip_transform, dino_transform
    from visreps_amd.models.foundation import CLIP_MEAN, CLIP_STD

    imgs = [_img(h, w, 40 + s) for s in range(2)]
    got = clip_transform().batch(imgs).cpu().numpy()
    for i, im in enumerate(imgs):
        assert np.array_equal(got[i], _pil_ref(im, 224, 224, CLIP_MEAN, CLIP_STD, "bicubic"))
    got = dino_transform().batch(imgs).cpu().numpy()
    for i, im in enumerate(imgs):
        assert np.array_equal(got[i], _pil_ref(im, 224, 224, DS_MEAN["imgnet"], DS_STD["imgnet"], "bicubic"))
