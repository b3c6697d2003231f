"""Image transforms (reference: python/paddle/vision/transforms/{transforms,functional}.py).
Operate on HWC numpy arrays / PIL images (host-side, inside DataLoader workers) and on CHW
paddle Tensors."""
from __future__ import annotations

import math
import numbers
import random

import numpy as np

from ..framework.core import Tensor, _wrap

__all__ = ["BaseTransform", "Compose", "Resize", "RandomResizedCrop", "CenterCrop", "RandomHorizontalFlip",
           "RandomVerticalFlip", "Transpose", "Normalize", "BrightnessTransform", "SaturationTransform",
           "ContrastTransform", "HueTransform", "ColorJitter", "RandomCrop", "Pad", "RandomAffine", "RandomRotation",
           "RandomPerspective", "Grayscale", "ToTensor", "RandomErasing", "to_tensor", "hflip", "vflip", "resize",
           "pad", "affine", "rotate", "perspective", "to_grayscale", "crop", "center_crop", "adjust_brightness",
           "adjust_contrast", "adjust_hue", "normalize", "erase", "adjust_saturation"]


def _is_pil(img):
    try:
        from PIL import Image
        return isinstance(img, Image.Image)
    except ImportError:
        return False


def _to_np(img):
    if _is_pil(img):
        return np.asarray(img)
    if isinstance(img, Tensor):
        return img.numpy()
    return np.asarray(img)


def _like(orig, arr):
    if _is_pil(orig):
        from PIL import Image
        return Image.fromarray(arr.astype(np.uint8) if arr.dtype != np.uint8 else arr)
    if isinstance(orig, Tensor):
        import torch
        return _wrap(torch.from_numpy(np.ascontiguousarray(arr)))
    return arr


def _size(img):
    a = _to_np(img)
    if isinstance(img, Tensor):
        return a.shape[-1], a.shape[-2]
    return a.shape[1], a.shape[0]


# ------------------------------------------------------------------------- functional
def to_tensor(pic, data_format="CHW"):
    import torch
    a = _to_np(pic)
    if a.ndim == 2:
        a = a[:, :, None]
    a = a.astype(np.float32) / 255.0 if a.dtype == np.uint8 else a.astype(np.float32)
    if data_format == "CHW":
        a = a.transpose(2, 0, 1)
    return _wrap(torch.from_numpy(np.ascontiguousarray(a)))


def hflip(img):
    if isinstance(img, Tensor):
        return _like(img, _to_np(img)[..., ::-1].copy())
    return _like(img, _to_np(img)[:, ::-1].copy())


def vflip(img):
    if isinstance(img, Tensor):
        return _like(img, _to_np(img)[..., ::-1, :].copy())
    return _like(img, _to_np(img)[::-1].copy())


def _resize_np(a, h, w, interpolation="bilinear"):
    from PIL import Image
    mode = {"nearest": Image.NEAREST, "bilinear": Image.BILINEAR, "bicubic": Image.BICUBIC,
            "lanczos": Image.LANCZOS, "box": Image.BOX, "hamming": Image.HAMMING}[interpolation]
    if a.dtype == np.uint8:
        if a.ndim == 3 and a.shape[2] == 1:
            return np.asarray(Image.fromarray(a[:, :, 0]).resize((w, h), mode))[:, :, None]
        return np.asarray(Image.fromarray(a).resize((w, h), mode))
    import torch
    import torch.nn.functional as TF
    t = torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32))
    t = t.permute(2, 0, 1)[None] if t.dim() == 3 else t[None, None]
    m = "bilinear" if interpolation in ("bilinear", "lanczos", "hamming", "box") else interpolation
    out = TF.interpolate(t, (h, w), mode=m, align_corners=False if m != "nearest" else None)
    out = out[0].permute(1, 2, 0).numpy() if a.ndim == 3 else out[0, 0].numpy()
    return out.astype(a.dtype)


def resize(img, size, interpolation="bilinear"):
    w, h = _size(img)
    if isinstance(size, int):
        if w < h:
            ow, oh = size, int(size * h / w)
        else:
            oh, ow = size, int(size * w / h)
    else:
        oh, ow = size
    if isinstance(img, Tensor):
        import torch.nn.functional as TF
        t = img._t
        out = TF.interpolate(t[None].float(), (oh, ow), mode="bilinear" if interpolation != "nearest" else "nearest")
        return _wrap(out[0].to(t.dtype))
    return _like(img, _resize_np(_to_np(img), oh, ow, interpolation))


def crop(img, top, left, height, width):
    if isinstance(img, Tensor):
        return _wrap(img._t[..., top:top + height, left:left + width])
    return _like(img, _to_np(img)[top:top + height, left:left + width])


def center_crop(img, output_size):
    if isinstance(output_size, numbers.Number):
        output_size = (int(output_size), int(output_size))
    w, h = _size(img)
    th, tw = output_size
    return crop(img, int(round((h - th) / 2.0)), int(round((w - tw) / 2.0)), th, tw)


def pad(img, padding, fill=0, padding_mode="constant"):
    if isinstance(padding, numbers.Number):
        padding = (padding,) * 4
    elif len(padding) == 2:
        padding = (padding[0], padding[1], padding[0], padding[1])
    l, t, r, b = padding
    a = _to_np(img)
    mode = {"constant": "constant", "edge": "edge", "reflect": "reflect", "symmetric": "symmetric"}[padding_mode]
    if isinstance(img, Tensor):
        pw = ((0, 0),) * (a.ndim - 2) + ((t, b), (l, r))
    else:
        pw = ((t, b), (l, r)) + ((0, 0),) * (a.ndim - 2)
    kw = {"constant_values": fill} if mode == "constant" else {}
    return _like(img, np.pad(a, pw, mode=mode, **kw))


def normalize(img, mean, std, data_format="CHW", to_rgb=False):
    if isinstance(img, Tensor):
        import torch
        t = img._t.float()
        shape = [-1, 1, 1] if data_format == "CHW" else [1, 1, -1]
        m = torch.tensor(mean, dtype=torch.float32, device=t.device).reshape(shape)
        s = torch.tensor(std, dtype=torch.float32, device=t.device).reshape(shape)
        return _wrap((t - m) / s)
    a = _to_np(img).astype(np.float32)
    if to_rgb:
        a = a[..., ::-1]
    shape = (-1, 1, 1) if data_format == "CHW" else (1, 1, -1)
    return (a - np.asarray(mean, np.float32).reshape(shape)) / np.asarray(std, np.float32).reshape(shape)


def to_grayscale(img, num_output_channels=1):
    a = _to_np(img).astype(np.float32)
    g = a[..., 0] * 0.299 + a[..., 1] * 0.587 + a[..., 2] * 0.114
    g = np.repeat(g[..., None], num_output_channels, -1)
    return _like(img, g.astype(_to_np(img).dtype))


def adjust_brightness(img, brightness_factor):
    a = _to_np(img).astype(np.float32) * brightness_factor
    return _like(img, np.clip(a, 0, 255).astype(_to_np(img).dtype))


def adjust_contrast(img, contrast_factor):
    a = _to_np(img).astype(np.float32)
    m = (a[..., 0] * 0.299 + a[..., 1] * 0.587 + a[..., 2] * 0.114).mean() if a.ndim == 3 else a.mean()
    return _like(img, np.clip((a - m) * contrast_factor + m, 0, 255).astype(_to_np(img).dtype))


def adjust_saturation(img, saturation_factor):
    a = _to_np(img).astype(np.float32)
    g = (a[..., 0] * 0.299 + a[..., 1] * 0.587 + a[..., 2] * 0.114)[..., None]
    return _like(img, np.clip((a - g) * saturation_factor + g, 0, 255).astype(_to_np(img).dtype))


def adjust_hue(img, hue_factor):
    import colorsys
    a = _to_np(img).astype(np.float32) / 255.0
    flat = a.reshape(-1, 3)
    hsv = np.array([colorsys.rgb_to_hsv(*p) for p in flat])
    hsv[:, 0] = (hsv[:, 0] + hue_factor) % 1.0
    rgb = np.array([colorsys.hsv_to_rgb(*p) for p in hsv]).reshape(a.shape)
    return _like(img, (rgb * 255).astype(_to_np(img).dtype))


def _affine_np(a, matrix, interpolation="nearest", fill=0):
    from PIL import Image
    im = Image.fromarray(a)
    resample = Image.NEAREST if interpolation == "nearest" else Image.BILINEAR
    return np.asarray(im.transform(im.size, Image.AFFINE, matrix, resample, fillcolor=fill))


def affine(img, angle, translate, scale, shear, interpolation="nearest", fill=0, center=None):
    w, h = _size(img)
    cx, cy = center if center is not None else (w * 0.5, h * 0.5)
    rot = math.radians(angle)
    sx, sy = [math.radians(s) for s in (shear if isinstance(shear, (list, tuple)) else (shear, 0.0))]
    a = math.cos(rot - sy) / math.cos(sy)
    b = -math.cos(rot - sy) * math.tan(sx) / math.cos(sy) - math.sin(rot)
    c = math.sin(rot - sy) / math.cos(sy)
    d = -math.sin(rot - sy) * math.tan(sx) / math.cos(sy) + math.cos(rot)
    M = np.array([[d, -b, 0], [-c, a, 0]]) / (scale * (a * d - b * c))
    tx, ty = translate
    M[0, 2] = M[0, 0] * (-cx - tx) + M[0, 1] * (-cy - ty) + cx
    M[1, 2] = M[1, 0] * (-cx - tx) + M[1, 1] * (-cy - ty) + cy
    return _like(img, _affine_np(_to_np(img), tuple(M.reshape(-1)), interpolation, fill))


def rotate(img, angle, interpolation="nearest", expand=False, center=None, fill=0):
    from PIL import Image
    a = _to_np(img)
    im = Image.fromarray(a)
    resample = Image.NEAREST if interpolation == "nearest" else Image.BILINEAR
    return _like(img, np.asarray(im.rotate(angle, resample, expand, center, fillcolor=fill)))


def perspective(img, startpoints, endpoints, interpolation="nearest", fill=0):
    from PIL import Image
    A, B = [], []
    for (x, y), (u, v) in zip(endpoints, startpoints):
        A.append([x, y, 1, 0, 0, 0, -u * x, -u * y])
        A.append([0, 0, 0, x, y, 1, -v * x, -v * y])
        B += [u, v]
    coeffs = np.linalg.lstsq(np.array(A, dtype=np.float64), np.array(B, dtype=np.float64), rcond=None)[0]
    im = Image.fromarray(_to_np(img))
    resample = Image.NEAREST if interpolation == "nearest" else Image.BILINEAR
    return _like(img, np.asarray(im.transform(im.size, Image.PERSPECTIVE, tuple(coeffs), resample, fillcolor=fill)))


def erase(img, i, j, h, w, v, inplace=False):
    if isinstance(img, Tensor):
        t = img._t if inplace else img._t.clone()
        t[..., i:i + h, j:j + w] = v._t if isinstance(v, Tensor) else v
        return img if inplace else _wrap(t)
    a = _to_np(img) if inplace else _to_np(img).copy()
    a[i:i + h, j:j + w] = v
    return _like(img, a)


# ------------------------------------------------------------------------- classes
class BaseTransform:
    def __init__(self, keys=None):
        self.keys = keys or ("image",)

    def __call__(self, inputs):
        if isinstance(inputs, tuple):
            return (self._apply_image(inputs[0]),) + tuple(inputs[1:])
        return self._apply_image(inputs)

    def _apply_image(self, img):
        raise NotImplementedError


class Compose:
    def __init__(self, transforms):
        self.transforms = transforms

    def __call__(self, data):
        for f in self.transforms:
            data = f(data)
        return data


class Resize(BaseTransform):
    def __init__(self, size, interpolation="bilinear", keys=None):
        super().__init__(keys)
        self.size, self.interpolation = size, interpolation

    def _apply_image(self, img):
        return resize(img, self.size, self.interpolation)


class RandomResizedCrop(BaseTransform):
    def __init__(self, size, scale=(0.08, 1.0), ratio=(3.0 / 4, 4.0 / 3), interpolation="bilinear", keys=None):
        super().__init__(keys)
        self.size = (size, size) if isinstance(size, int) else size
        self.scale, self.ratio, self.interpolation = scale, ratio, interpolation

    def _params(self, img):
        w, h = _size(img)
        area = w * h
        for _ in range(10):
            ta = random.uniform(*self.scale) * area
            ar = math.exp(random.uniform(math.log(self.ratio[0]), math.log(self.ratio[1])))
            cw, ch = int(round(math.sqrt(ta * ar))), int(round(math.sqrt(ta / ar)))
            if 0 < cw <= w and 0 < ch <= h:
                return random.randint(0, h - ch), random.randint(0, w - cw), ch, cw
        s = min(w, h)
        return (h - s) // 2, (w - s) // 2, s, s

    def _apply_image(self, img):
        i, j, h, w = self._params(img)
        return resize(crop(img, i, j, h, w), self.size, self.interpolation)


class CenterCrop(BaseTransform):
    def __init__(self, size, keys=None):
        super().__init__(keys)
        self.size = size

    def _apply_image(self, img):
        return center_crop(img, self.size)


class RandomHorizontalFlip(BaseTransform):
    def __init__(self, prob=0.5, keys=None):
        super().__init__(keys)
        self.prob = prob

    def _apply_image(self, img):
        return hflip(img) if random.random() < self.prob else img


class RandomVerticalFlip(BaseTransform):
    def __init__(self, prob=0.5, keys=None):
        super().__init__(keys)
        self.prob = prob

    def _apply_image(self, img):
        return vflip(img) if random.random() < self.prob else img


class Normalize(BaseTransform):
    def __init__(self, mean=0.0, std=1.0, data_format="CHW", to_rgb=False, keys=None):
        super().__init__(keys)
        self.mean = [mean] * 3 if isinstance(mean, numbers.Number) else mean
        self.std = [std] * 3 if isinstance(std, numbers.Number) else std
        self.data_format, self.to_rgb = data_format, to_rgb

    def _apply_image(self, img):
        return normalize(img, self.mean, self.std, self.data_format, self.to_rgb)


class Transpose(BaseTransform):
    def __init__(self, order=(2, 0, 1), keys=None):
        super().__init__(keys)
        self.order = order

    def _apply_image(self, img):
        if isinstance(img, Tensor):
            return _wrap(img._t.permute(*self.order))
        a = _to_np(img)
        if a.ndim == 2:
            a = a[..., None]
        return a.transpose(self.order)


class BrightnessTransform(BaseTransform):
    def __init__(self, value, keys=None):
        super().__init__(keys)
        self.value = value

    def _apply_image(self, img):
        return adjust_brightness(img, random.uniform(max(0, 1 - self.value), 1 + self.value)) if self.value else img


class ContrastTransform(BaseTransform):
    def __init__(self, value, keys=None):
        super().__init__(keys)
        self.value = value

    def _apply_image(self, img):
        return adjust_contrast(img, random.uniform(max(0, 1 - self.value), 1 + self.value)) if self.value else img


class SaturationTransform(BaseTransform):
    def __init__(self, value, keys=None):
        super().__init__(keys)
        self.value = value

    def _apply_image(self, img):
        return adjust_saturation(img, random.uniform(max(0, 1 - self.value), 1 + self.value)) if self.value else img


class HueTransform(BaseTransform):
    def __init__(self, value, keys=None):
        super().__init__(keys)
        self.value = value

    def _apply_image(self, img):
        return adjust_hue(img, random.uniform(-self.value, self.value)) if self.value else img


class ColorJitter(BaseTransform):
    def __init__(self, brightness=0, contrast=0, saturation=0, hue=0, keys=None):
        super().__init__(keys)
        self.ts = [BrightnessTransform(brightness), ContrastTransform(contrast), SaturationTransform(saturation),
                   HueTransform(hue)]

    def _apply_image(self, img):
        random.shuffle(self.ts)
        for t in self.ts:
            img = t._apply_image(img)
        return img


class RandomCrop(BaseTransform):
    def __init__(self, size, padding=None, pad_if_needed=False, fill=0, padding_mode="constant", keys=None):
        super().__init__(keys)
        self.size = (size, size) if isinstance(size, int) else size
        self.padding, self.pad_if_needed, self.fill, self.padding_mode = padding, pad_if_needed, fill, padding_mode

    def _apply_image(self, img):
        if self.padding is not None:
            img = pad(img, self.padding, self.fill, self.padding_mode)
        w, h = _size(img)
        th, tw = self.size
        if self.pad_if_needed and w < tw:
            img = pad(img, (tw - w, 0), self.fill, self.padding_mode)
        if self.pad_if_needed and h < th:
            img = pad(img, (0, th - h), self.fill, self.padding_mode)
        w, h = _size(img)
        i = random.randint(0, h - th)
        j = random.randint(0, w - tw)
        return crop(img, i, j, th, tw)


class Pad(BaseTransform):
    def __init__(self, padding, fill=0, padding_mode="constant", keys=None):
        super().__init__(keys)
        self.padding, self.fill, self.padding_mode = padding, fill, padding_mode

    def _apply_image(self, img):
        return pad(img, self.padding, self.fill, self.padding_mode)


class RandomAffine(BaseTransform):
    def __init__(self, degrees, translate=None, scale=None, shear=None, interpolation="nearest", fill=0, center=None, keys=None):
        super().__init__(keys)
        self.degrees = (-degrees, degrees) if isinstance(degrees, numbers.Number) else degrees
        self.translate, self.scale, self.shear = translate, scale, shear
        self.interpolation, self.fill, self.center = interpolation, fill, center

    def _apply_image(self, img):
        w, h = _size(img)
        angle = random.uniform(*self.degrees)
        tr = (0, 0)
        if self.translate is not None:
            tr = (int(round(random.uniform(-self.translate[0] * w, self.translate[0] * w))),
                  int(round(random.uniform(-self.translate[1] * h, self.translate[1] * h))))
        sc = random.uniform(*self.scale) if self.scale is not None else 1.0
        sh = (0.0, 0.0)
        if self.shear is not None:
            s = (-self.shear, self.shear) if isinstance(self.shear, numbers.Number) else self.shear
            sh = (random.uniform(s[0], s[1]), random.uniform(s[2], s[3]) if len(s) == 4 else 0.0)
        return affine(img, angle, tr, sc, sh, self.interpolation, self.fill, self.center)


class RandomRotation(BaseTransform):
    def __init__(self, degrees, interpolation="nearest", expand=False, center=None, fill=0, keys=None):
        super().__init__(keys)
        self.degrees = (-degrees, degrees) if isinstance(degrees, numbers.Number) else degrees
        self.interpolation, self.expand, self.center, self.fill = interpolation, expand, center, fill

    def _apply_image(self, img):
        return rotate(img, random.uniform(*self.degrees), self.interpolation, self.expand, self.center, self.fill)


class RandomPerspective(BaseTransform):
    def __init__(self, prob=0.5, distortion_scale=0.5, interpolation="nearest", fill=0, keys=None):
        super().__init__(keys)
        self.prob, self.distortion_scale, self.interpolation, self.fill = prob, distortion_scale, interpolation, fill

    def _apply_image(self, img):
        if random.random() >= self.prob:
            return img
        w, h = _size(img)
        hw, hh = int(self.distortion_scale * w / 2), int(self.distortion_scale * h / 2)
        start = [[0, 0], [w - 1, 0], [w - 1, h - 1], [0, h - 1]]
        end = [[random.randint(0, hw), random.randint(0, hh)], [w - 1 - random.randint(0, hw), random.randint(0, hh)],
               [w - 1 - random.randint(0, hw), h - 1 - random.randint(0, hh)], [random.randint(0, hw), h - 1 - random.randint(0, hh)]]
        return perspective(img, start, end, self.interpolation, self.fill)


class Grayscale(BaseTransform):
    def __init__(self, num_output_channels=1, keys=None):
        super().__init__(keys)
        self.n = num_output_channels

    def _apply_image(self, img):
        return to_grayscale(img, self.n)


class ToTensor(BaseTransform):
    def __init__(self, data_format="CHW", keys=None):
        super().__init__(keys)
        self.data_format = data_format

    def _apply_image(self, img):
        return to_tensor(img, self.data_format)


class RandomErasing(BaseTransform):
    def __init__(self, prob=0.5, scale=(0.02, 0.33), ratio=(0.3, 3.3), value=0, inplace=False, keys=None):
        super().__init__(keys)
        self.prob, self.scale, self.ratio, self.value, self.inplace = prob, scale, ratio, value, inplace

    def _apply_image(self, img):
        if random.random() >= self.prob:
            return img
        a = _to_np(img)
        h, w = (a.shape[-2], a.shape[-1]) if isinstance(img, Tensor) else a.shape[:2]
        for _ in range(10):
            ea = random.uniform(*self.scale) * h * w
            ar = math.exp(random.uniform(math.log(self.ratio[0]), math.log(self.ratio[1])))
            eh, ew = int(round(math.sqrt(ea * ar))), int(round(math.sqrt(ea / ar)))
            if eh < h and ew < w:
                return erase(img, random.randint(0, h - eh), random.randint(0, w - ew), eh, ew, self.value, self.inplace)
        return img
