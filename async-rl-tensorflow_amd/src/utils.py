"""Small helpers the reference keeps in src/utils.py:1-15.

``timeit`` wraps a callable and prints its wall time in the reference's format
("   [-] <name> : <seconds> sec"); ``get_time`` is the UTC timestamp string the reference
uses for monitor directories ("YYYY-mm-dd_HH:MM:SS").
"""
import functools
import time

_STAMP = '%Y-%m-%d_%H:%M:%S'


def timeit(fn):
  @functools.wraps(fn)
  def wrapper(*args, **kwargs):
    t0 = time.time()
    try:
      return fn(*args, **kwargs)
    finally:
      print('   [-] {} : {:2.5f} sec'.format(fn.__name__, time.time() - t0))
  return wrapper


def get_time():
  return time.strftime(_STAMP, time.gmtime())
