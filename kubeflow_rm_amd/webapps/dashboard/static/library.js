/**
 * Central dashboard <-> iframed app protocol (same message contract as the reference
 * centraldashboard/public/library.js): the dashboard posts `parent-connected`, then
 * `namespace-selected` {value: ns} / `all-namespaces` {value: [...]}; the app answers
 * `iframe-connected`. Usage: window.centraldashboard.CentralDashboardEventHandler.init(cb).
 */
(function (global) {
  "use strict";
  const EV = { PARENT_CONNECTED: "parent-connected", APP_CONNECTED: "iframe-connected",
               NAMESPACE_SELECTED: "namespace-selected", ALL_NAMESPACES: "all-namespaces" };
  class Handler {
    constructor() { this.onParentConnected = null; this.onNamespaceSelected = null; this.onAllNamespacesSelected = null; this._l = null; }
    get isIframed() { return window.location !== window.parent.location; }
    get isOpenedByApp() { return window.opener !== null && window.opener !== undefined; }
    init(callback, disableForceIframe = false) {
      callback(this, this.isIframed || this.isOpenedByApp);
      if (this.isOpenedByApp || this.isIframed) {
        this._l = (ev) => this._dispatch(ev.data || {});
        window.addEventListener("message", this._l);
        (this.isIframed ? window.parent : window.opener).postMessage({ type: EV.APP_CONNECTED }, "*");
      } else if (!disableForceIframe) {
        fetch("/api/dashboard-settings").then((r) => r.json()).then((d) => {
          if (d.DASHBOARD_FORCE_IFRAME) window.location.replace(window.location.origin + "/_" + window.location.pathname + window.location.search);
        }).catch((e) => console.error(e));
      }
    }
    detach() { if (this._l) window.removeEventListener("message", this._l); this._l = null; }
    _dispatch(d) {
      if (d.type === EV.PARENT_CONNECTED && this.onParentConnected) this.onParentConnected(d);
      if (d.type === EV.NAMESPACE_SELECTED && this.onNamespaceSelected) this.onNamespaceSelected(d.value);
      if (d.type === EV.ALL_NAMESPACES && this.onAllNamespacesSelected) this.onAllNamespacesSelected(d.value);
    }
  }
  global.centraldashboard = { CentralDashboardEventHandler: new Handler(), EVENTS: EV };
})(window);
