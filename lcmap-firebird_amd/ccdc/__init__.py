"""``ccdc`` -- mirror of lcmap-firebird's ``ccdc`` package restricted to the change-detection
hot path: ``ccdc.pyccd`` (the plugin boundary), ``ccdc.segment`` / ``pixel`` /
``chip`` (output schemas and projections) and ``ccdc.timeseries`` (the ARD record layout and a
chip packer).  The reference ``ccdc/__init__.py:11-76`` reads cluster env vars and builds a
SparkContext at import time; that control plane is out of scope, so only the logger helper is
kept (``ccdc/__init__.py:64-76``), backed by the standard ``logging`` module.
"""
import logging
import multiprocessing
import os

PRODUCT_PARTITIONS = int(os.environ.get('PRODUCT_PARTITIONS', multiprocessing.cpu_count() * 8))


def logger(context=None, name=None):
    """ccdc.logger(context, name) -> a logger (log4j through py4j in the reference)."""
    return logging.getLogger(name or 'ccdc')
