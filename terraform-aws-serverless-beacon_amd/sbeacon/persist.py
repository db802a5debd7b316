"""A set of persisted stores, rebuilt per group only when its VCFs changed.

The reference keeps its ingest state between invocations -- each VCF's
region files in S3 (lambda/summariseSlice/source/write_data_to_s3.h:39-92)
and the dataset's toUpdate bookkeeping in DynamoDB
(lambda/summariseSlice/source/main.cpp:360-438) -- and summariseVcf only
re-summarises the files that changed.  Here a deployment keeps its VCFs as
groups (a dataset, or one VCF), one store per group under ``root/<group>``
(sb_store_save).  ``StoreSet.load`` opens every saved group whose source
files are unchanged (sb_store_open: no VCF re-read) and re-ingests only the
groups that are missing or stale, saving them again.
"""
from __future__ import annotations

import os
import shutil

from .engine import StaleStore, Store


class StoreSet:
    def __init__(self, root: str):
        self.root = root
        self.stores: dict[str, Store] = {}
        self.rebuilt: list[str] = []  # groups ingested by the last load()
        self.opened: list[str] = []   # groups re-opened from disk

    def load(self, groups: dict, *, device: int = 0, keep_genotypes: bool = True, n_threads: int = 0) -> dict:
        """``groups``: name -> [(vcf_location, path), ...].  Returns name -> Store."""
        os.makedirs(self.root, exist_ok=True)
        self.rebuilt, self.opened = [], []
        for name, sources in groups.items():
            d = os.path.join(self.root, name)
            st = None
            if os.path.exists(os.path.join(d, 'manifest.json')):
                try:
                    st = Store.open(d, device=device)
                    want = {loc: os.path.abspath(os.fspath(p)) for loc, p in sources}
                    have = {loc: os.path.abspath(os.fspath(p)) for loc, p in st.paths.items()}
                    if sorted(st.locations) != sorted(want) or have != want:
                        # the group's membership changed, or a location now
                        # names another file (the saved fingerprints are of
                        # the old files, which may well be unchanged)
                        st.close()
                        st = None
                    else:
                        self.opened.append(name)
                except StaleStore:
                    st = None
            if st is None:
                st = Store.build(sources, device=device, keep_genotypes=keep_genotypes, n_threads=n_threads)
                tmp = d + '.tmp'
                shutil.rmtree(tmp, ignore_errors=True)
                st.save(tmp)
                shutil.rmtree(d, ignore_errors=True)
                os.replace(tmp, d)
                self.rebuilt.append(name)
            self.stores[name] = st
        return self.stores
