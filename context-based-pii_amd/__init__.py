"""MI355X-native PII scan-and-redact engine (drop-in for call_dlp_for_redaction's deidentify step).

The directory name is not a Python identifier; import it with
``importlib.import_module("context-based-pii_amd")`` (see ``pii_amd.load()``).
"""
