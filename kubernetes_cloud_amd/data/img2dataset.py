"""Image-text dataset downloader (spark/docker/download_imgdataset.py).

Same CLI as the reference job (``--url-list`` parquet with URL / TEXT columns,
``--output``, ``--thread-count``) and the same output contract as
``img2dataset(output_format="webdataset", image_size=256, subjob_size=1000)``:
``{output}/{shard:05d}.tar`` shards holding ``{key}.jpg`` (resized to
``image_size`` with a centre pad, the img2dataset "border" mode), ``{key}.txt``
(caption) and ``{key}.json`` (url, caption, status, original size), plus a
``{shard:05d}_stats.json`` per shard.

Distribution: when ``pyspark`` and ``img2dataset`` are importable (the Spark
image of spark/example-spark-submit.sh) the job delegates to them with
``distributor="pyspark"`` exactly like the reference; otherwise shards are
processed by a local process pool with a thread pool per shard. CPU only.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import io
import json
import os
import tarfile
import time


def _resize(data: bytes, size: int) -> tuple[bytes, tuple[int, int]]:
    from PIL import Image

    im = Image.open(io.BytesIO(data)).convert("RGB")
    orig = im.size
    scale = size / max(orig)
    im = im.resize((max(1, round(orig[0] * scale)), max(1, round(orig[1] * scale))), Image.BICUBIC)
    canvas = Image.new("RGB", (size, size), (255, 255, 255))
    canvas.paste(im, ((size - im.size[0]) // 2, (size - im.size[1]) // 2))
    out = io.BytesIO()
    canvas.save(out, format="JPEG", quality=95)
    return out.getvalue(), orig


def _fetch(url: str, timeout: float) -> bytes:
    import requests

    r = requests.get(url, timeout=timeout)
    r.raise_for_status()
    return r.content


def _add(tar: tarfile.TarFile, name: str, payload: bytes):
    info = tarfile.TarInfo(name)
    info.size = len(payload)
    info.mtime = int(time.time())
    tar.addfile(info, io.BytesIO(payload))


def process_shard(shard: int, rows: list[tuple[str, str]], output: str, image_size: int, threads: int,
                  timeout: float = 10.0) -> dict:
    t0 = time.time()
    ok = fail = 0
    path = os.path.join(output, f"{shard:05d}.tar")
    with cf.ThreadPoolExecutor(max_workers=max(1, threads)) as ex:
        futs = [ex.submit(_fetch, u, timeout) for u, _ in rows]
        with tarfile.open(path + ".tmp", "w") as tar:
            for i, ((url, cap), fut) in enumerate(zip(rows, futs)):
                key = f"{shard:05d}{i:04d}"
                meta = {"url": url, "caption": cap, "key": key}
                try:
                    img, orig = _resize(fut.result(), image_size)
                    meta.update(status="success", original_width=orig[0], original_height=orig[1])
                    _add(tar, key + ".jpg", img)
                    _add(tar, key + ".txt", (cap or "").encode())
                    _add(tar, key + ".json", json.dumps(meta).encode())
                    ok += 1
                except Exception as e:  # noqa: BLE001 - per-sample failures are data, as in img2dataset
                    meta.update(status="failed_to_download", error_message=str(e)[:200])
                    fail += 1
    os.replace(path + ".tmp", path)
    stats = {"shard": shard, "count": len(rows), "successes": ok, "failed_to_download": fail,
             "duration": round(time.time() - t0, 3)}
    with open(os.path.join(output, f"{shard:05d}_stats.json"), "w") as f:
        json.dump(stats, f)
    return stats


def download(url_list: str, output: str, thread_count: int = 16, image_size: int = 256, subjob_size: int = 1000,
             url_col: str = "URL", caption_col: str = "TEXT", processes: int | None = None) -> list[dict]:
    try:  # the reference's distributed path
        import img2dataset  # noqa: F401
        import pyspark  # noqa: F401
        from img2dataset import download as i2d

        i2d(thread_count=thread_count, url_list=url_list, image_size=image_size, output_folder=output,
            output_format="webdataset", input_format="parquet", url_col=url_col, caption_col=caption_col,
            subjob_size=subjob_size, distributor="pyspark")
        return []
    except ImportError:
        pass
    import pyarrow.parquet as pq

    tbl = pq.read_table(url_list, columns=[url_col, caption_col])
    urls = tbl.column(url_col).to_pylist()
    caps = tbl.column(caption_col).to_pylist()
    rows = list(zip(urls, caps))
    os.makedirs(output, exist_ok=True)
    shards = [rows[i:i + subjob_size] for i in range(0, len(rows), subjob_size)]
    procs = processes or min(len(shards), os.cpu_count() or 1) or 1
    per = max(1, thread_count // procs)
    if procs == 1:
        return [process_shard(i, s, output, image_size, per) for i, s in enumerate(shards)]
    with cf.ProcessPoolExecutor(max_workers=procs) as ex:
        return list(ex.map(process_shard, range(len(shards)), shards, [output] * len(shards),
                           [image_size] * len(shards), [per] * len(shards)))


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--url-list", default="/mnt/pvc/mscoco.parquet", help="Path to the url list file")
    ap.add_argument("--output", default="/mnt/pvc/mscoco", help="Path to output folder")
    ap.add_argument("--thread-count", "-t", type=int, default=16, help="Number of download threads")
    ap.add_argument("--image-size", type=int, default=256)
    ap.add_argument("--subjob-size", type=int, default=1000)
    ap.add_argument("--processes", type=int, default=None)
    a = ap.parse_args(argv)
    if not os.path.exists(a.url_list):
        raise ValueError(f"The URL list does not exist at: {a.url_list}")
    stats = download(a.url_list, a.output, a.thread_count, a.image_size, a.subjob_size, processes=a.processes)
    ok = sum(s["successes"] for s in stats)
    print(json.dumps({"shards": len(stats), "successes": ok, "total": sum(s["count"] for s in stats)}))


if __name__ == "__main__":
    main()
