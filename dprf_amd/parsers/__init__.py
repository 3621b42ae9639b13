"""Python-3 counterparts of the reference's document parsers (L3 in SURVEY.md section 1).

Each one prints/returns the same ``name:$fmt$*field*...`` line as the reference parser run under
Python 2, so the streams fed to the verification engine are
byte-identical.  They are host-side, run once per document, and never touch the GPU.
"""
