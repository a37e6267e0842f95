"""pygame stand-in: only the name `Surface` is evaluated at class-definition time."""


class Surface:
    pass
