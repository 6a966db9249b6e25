"""rspl_slam_amd -- MI355X-native SuperPoint -> SuperGlue -> local-BA hot path.

Import via ``rspl_loader.load()`` (the directory name carries a dash, so it is
loaded by path as the module ``rspl_slam_amd``).
"""
