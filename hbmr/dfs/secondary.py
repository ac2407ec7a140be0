"""SecondaryNameNode: periodic offline checkpoint of the NameNode's metadata.

Behaviour from hadoop-1.0.3/src/hdfs/org/apache/hadoop/hdfs/server/namenode/
SecondaryNameNode.java: every ``fs.checkpoint.period`` seconds, or sooner once
the edit log exceeds ``fs.checkpoint.size`` bytes, it asks the NameNode to roll
its edit log (rollEditLog), downloads fsimage + the rolled edits
(GetImageServlet), merges them in ``fs.checkpoint.dir`` and uploads the new
image (rollFsImage), so the NameNode's edit log never grows without bound and
start-up replays only the edits since the last checkpoint.

The NameNode here is reached either in-process or over hbmr RPC; the
"download/upload" are plain method calls returning/accepting the JSON image.
Segment ids make the merge crash-safe: an image records the last edit
segment merged into it, so a crash between roll and install never replays a
segment twice (see NameNode._load).
"""
from __future__ import annotations

import json
import logging
import os
import shutil
import threading

from .namenode import NameNode

log = logging.getLogger("hbmr.dfs.secondary")


class SecondaryNameNode:
    def __init__(self, namenode, checkpoint_dir, conf=None, period_s=None, size_bytes=None,
                 name_dir=None):
        self.nn = namenode
        self.dir = checkpoint_dir
        self.name_dir = name_dir
        self.period = period_s if period_s is not None else \
            (conf.get_int("fs.checkpoint.period", 3600) if conf is not None else 3600)
        self.size = size_bytes if size_bytes is not None else \
            (conf.get_long("fs.checkpoint.size", 64 << 20) if conf is not None else 64 << 20)
        self.checkpoints = 0
        self._stop = threading.Event()
        self._thread = None
        os.makedirs(self.dir, exist_ok=True)

    def edits_size(self) -> int:
        if self.name_dir:
            p = os.path.join(self.name_dir, "edits")
            return os.path.getsize(p) if os.path.exists(p) else 0
        return 0

    def do_checkpoint(self) -> bool:
        """One roll → merge → install cycle."""
        rolled = self.nn.roll_edit_log()
        seg = rolled["segment"]
        files = self.nn.get_checkpoint_files()
        work = os.path.join(self.dir, "current")
        shutil.rmtree(work, ignore_errors=True)
        os.makedirs(work)
        if files["image"]:
            with open(os.path.join(work, "fsimage.json"), "w") as f:
                f.write(files["image"])
        with open(os.path.join(work, "edits"), "w") as f:
            f.write(files["edits"])
        merged = NameNode(name_dir=work, checkpoint_only=True)
        image = json.dumps(merged._image(seg))
        with open(os.path.join(self.dir, "fsimage.json"), "w") as f:
            f.write(image)   # our own copy: the last good checkpoint
        self.nn.install_checkpoint(image, seg)
        self.checkpoints += 1
        log.info("checkpoint through edit segment %d installed", seg)
        return True

    def _run(self):
        import time
        last = time.time()
        while not self._stop.wait(min(1.0, max(self.period, 0.05))):
            if time.time() - last >= self.period or self.edits_size() >= self.size:
                try:
                    self.do_checkpoint()
                except Exception:  # noqa: BLE001
                    log.exception("checkpoint failed")
                last = time.time()

    def start(self):
        self._thread = threading.Thread(target=self._run, daemon=True, name="SecondaryNameNode")
        self._thread.start()
        return self

    def shutdown(self):
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=10)
