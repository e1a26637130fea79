"""Test-infrastructure oracle (CPU restatement of the reference hot path). Never imported by the
product package; see torch_ref.py's header."""
