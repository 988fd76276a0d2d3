"""Labelme polygon annotations -> semantic-segmentation dataset (imgs/ + masks/ + data.yaml).

Parity: reference utils/check_datasets.py:15-111.  Same behaviour -- read
``<root>/labels/*.json``, shuffle with seed 0, 95/5 train/val split, class ids
in order of first appearance (``_background`` = 0), PNG images and index masks
under ``<root>/out/{train,val}/{imgs,masks}``, and a ``data.yaml`` with
``path`` and ``names`` -- but without the ``labelme`` / ``cv2`` packages (not
installed here): the JSON is parsed directly, ``imageData`` is decoded with
PIL, and polygons are rasterised with ``PIL.ImageDraw`` (labelme's own
``shapes_to_label`` draws with ``ImageDraw.polygon(xy, outline=1, fill=1)``,
so masks are identical).  Images are written in RGB order (the reference
flips to BGR only to undo cv2's BGR writer; the PNG content matches).
"""
from __future__ import annotations

import argparse
import base64
import io
import json
import os
import random
import shutil

import numpy as np
from PIL import Image, ImageDraw


def load_labelme(path):
    with open(path, "r", encoding="utf-8") as f:
        data = json.load(f)
    if data.get("imageData"):
        img = Image.open(io.BytesIO(base64.b64decode(data["imageData"])))
    else:  # image stored next to the json
        img = Image.open(os.path.join(os.path.dirname(path), data["imagePath"]))
    img = np.asarray(img.convert("RGB") if img.mode not in ("L", "RGB") else img)
    return img, data.get("shapes", [])


def shapes_to_label(img_shape, shapes, label_name_to_value):
    """Polygon shapes -> int32 class mask (later shapes paint over earlier ones)."""
    h, w = img_shape[:2]
    cls = np.zeros((h, w), dtype=np.int32)
    for shape in shapes:
        if shape.get("shape_type", "polygon") not in ("polygon", None):
            continue
        name = shape.get("label", "None")
        if name not in label_name_to_value:
            continue
        m = Image.new("L", (w, h), 0)
        xy = [tuple(map(float, p)) for p in shape["points"]]
        if len(xy) >= 2:
            ImageDraw.Draw(m).polygon(xy=xy, outline=1, fill=1)
        cls[np.asarray(m, dtype=bool)] = label_name_to_value[name]
    return cls


def check_semantic_segmentation_datasets(datasets_path, train_factor=0.95, seed=0):
    labels_path = os.path.join(datasets_path, "labels")
    if not os.path.exists(labels_path):
        print(f"Error: {labels_path} not found")
        return None
    root = os.path.join(datasets_path, "out")
    dirs = {s: {k: os.path.join(root, s, k) for k in ("imgs", "masks")} for s in ("train", "val")}
    if os.path.exists(root):
        shutil.rmtree(root)
    for s in dirs.values():
        for d in s.values():
            os.makedirs(d, exist_ok=True)

    rng = random.Random(seed)
    all_data = sorted(i for i in os.listdir(labels_path) if os.path.splitext(i)[1] == ".json")
    print("all_data: ", len(all_data))
    rng.shuffle(all_data)
    train_num = round(train_factor * len(all_data))

    class_name_to_id = {"_background": 0}
    for name in all_data:
        _, shapes = _shapes_only(os.path.join(labels_path, name))
        for shape in shapes:
            if shape.get("shape_type", "") == "polygon":
                class_name_to_id.setdefault(shape.get("label", "None"), len(class_name_to_id))
    print(class_name_to_id)

    for split, items in (("train", all_data[:train_num]), ("val", all_data[train_num:])):
        for name in items:
            stem = os.path.splitext(os.path.basename(name))[0]
            img, shapes = load_labelme(os.path.join(labels_path, name))
            lbl = shapes_to_label(img.shape, shapes, class_name_to_id)
            Image.fromarray(img).save(os.path.join(dirs[split]["imgs"], stem + ".png"))
            Image.fromarray(lbl.astype(np.uint8 if lbl.max() < 256 else np.uint16)).save(
                os.path.join(dirs[split]["masks"], stem + ".png"))

    with open(os.path.join(root, "data.yaml"), "w", encoding="utf-8") as f:
        f.write(f"path: {os.path.abspath(root)}\n")
        f.write("names: \n")
        for k, v in sorted(class_name_to_id.items(), key=lambda kv: kv[1]):
            f.write(f"  {v}: {k}\n")
    return class_name_to_id


def _shapes_only(path):
    with open(path, "r", encoding="utf-8") as f:
        data = json.load(f)
    return data, data.get("shapes", [])


def parse_opt(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--datasets_root", type=str, default="", help="path to datasets root dir.")
    return p.parse_args(argv)


if __name__ == "__main__":
    check_semantic_segmentation_datasets(parse_opt().datasets_root)
