"""Service entry point: ``uvicorn main:app`` or ``python main.py`` (127.0.0.1:8000).

The application lives in :mod:`penroz.serve.app`; this module only re-exports it.
"""
from penroz.serve.app import app, model_locks, dataset_locks  # noqa: F401

if __name__ == "__main__":  # pragma: no cover
    from penroz.serve.app import main
    main()
