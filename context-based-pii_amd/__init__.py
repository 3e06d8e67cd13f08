"""MI355X-native PII scan-and-redact engine (drop-in for call_dlp_for_redaction's deidentify step).

The directory name is not a Python identifier; import its modules with
``importlib.import_module("context-based-pii_amd.engine")`` (``.service``, ``.app``, ...), as
``tests/conftest.py`` (``pkg``) and ``__graft_entry__.py`` (``_pkg``) do.
"""
