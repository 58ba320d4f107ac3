"""Directory helpers (reference utils/path.py:1-36)."""
import glob
import os


def get_immediate_subdirectories(input_dir):
    return sorted(name for name in os.listdir(input_dir)
                  if os.path.isdir(os.path.join(input_dir, name)))


def get_recursive_subdirectories(input_dir, ext):
    """Relative paths of every directory (recursively, including ``.``) that
    holds at least one ``*.ext`` file."""
    lines = glob.glob('%s/**/*.%s' % (input_dir, ext), recursive=True)
    dirs = set()
    for line in lines:
        rel = os.path.relpath(os.path.dirname(line), input_dir)
        dirs.add(rel)
    return sorted(dirs)
