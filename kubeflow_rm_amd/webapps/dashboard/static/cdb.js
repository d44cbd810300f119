/**
 * Central dashboard logic without the DOM: URL mirroring between the browser and the app iframe,
 * namespace selection, menu state, and the page renderers (HTML strings). app.js wires it to the
 * page; tests/js/test_dashboard.js drives it under node against the reference Cypress fixtures.
 *
 * Behaviour covered (reference, /root/reference/components/):
 *  - centraldashboard-angular/frontend/src/app/pages/iframe-wrapper/iframe-wrapper.component.ts:
 *    browser URL "/_/<app path>" <-> iframe URL "<app path>", polled every 100 ms, the namespace
 *    carried as ?ns= in the browser URL only, trailing slashes appended for Istio routes, the
 *    iframe not reloaded when the two URLs already agree (except for an explicit menu click).
 *  - .../services/namespace.service.ts: "All namespaces" only under jupyter/volumes/tensorboards/
 *    katib/models; selection priority ?ns= -> local storage -> first owned -> first valid.
 *  - .../guards/iframe.guard.ts: a menu link with an unresolved {ns} goes to namespace-needed.
 *  - centraldashboard/public/components/main-page.js: longest-prefix active menu item (hash- and
 *    path-based links), {ns} substitution; activities-list.js: day groups, newest first;
 *    registration-page.js: namespace-name rule and the 20 s profile poll.
 */
(function (root, factory) {
  if (typeof module === "object" && module.exports) module.exports = factory();
  else root.cdb = factory();
})(typeof self !== "undefined" ? self : this, function () {
  "use strict";

  const ALL_NAMESPACES = "All namespaces";
  const NO_NAMESPACES = "No namespaces";
  const ALL_NS_APPS = ["jupyter", "volumes", "tensorboards", "katib", "models"];
  const IFRAME_PREFIX = "/_";
  const BASE = "http://dashboard.invalid";  // URL parsing base; only path/search/hash are used

  const esc = (s) => String(s == null ? "" : s).replace(/[&<>"']/g, (c) =>
    ({ "&": "&amp;", "<": "&lt;", ">": "&gt;", '"': "&quot;", "'": "&#39;" }[c]));

  // ---- URLs ----------------------------------------------------------------------------------
  function parse(url) {
    const u = new URL(url || "/", BASE);
    return { path: u.pathname, search: u.search, hash: u.hash };
  }

  /** "/jupyter?x=1#f" -> "/jupyter/?x=1#f": apps behind Istio are routed on a trailing slash. */
  function withSlash(url) {
    const u = parse(url);
    return (u.path.endsWith("/") ? u.path : u.path + "/") + u.search + u.hash;
  }

  /** "/_/jupyter/" -> "/jupyter/" (the browser-side prefix of an iframed app). */
  function stripPrefix(url) {
    url = url || "";
    return url.startsWith(IFRAME_PREFIX + "/") || url === IFRAME_PREFIX ? url.slice(IFRAME_PREFIX.length) || "/" : url;
  }

  function queryParams(search) {
    const out = {};
    new URLSearchParams(search || "").forEach((v, k) => { out[k] = v; });
    return out;
  }

  function queryString(params) {
    const qs = new URLSearchParams(params).toString();
    return qs ? "?" + qs : "";
  }

  function fragmentOf(url) {
    const i = (url || "").indexOf("#");
    return i < 0 ? undefined : url.slice(i + 1);
  }

  /** Same page for the iframe: paths equal up to a trailing slash, same query without ns, same hash. */
  function sameUrl(a, b) {
    if (!a || !b) return false;
    const norm = (x) => {
      const u = parse(withSlash(x));
      const q = queryParams(u.search);
      delete q.ns;
      return u.path + queryString(q) + u.hash;
    };
    return norm(a) === norm(b);
  }

  // ---- namespaces ----------------------------------------------------------------------------
  function allNamespacesAllowed(url) {
    const p = stripPrefix(parse(url).path).replace(/^\/+/, "");
    return ALL_NS_APPS.some((app) => p === app || p.startsWith(app + "/"));
  }

  /** Selector options for a browser URL: the "All namespaces" entry first, disabled off its apps. */
  function namespaceOptions(namespaces, url) {
    return [{ namespace: ALL_NAMESPACES, role: "", user: "", disabled: !allNamespacesAllowed(url) },
            ...(namespaces || []).map((n) => ({ ...n, disabled: false }))];
  }

  function storageKey(user) {
    return "selectedNamespace/" + (user ? "." + user : "");
  }

  function usable(opt) {
    return !!opt && !(opt.namespace === ALL_NAMESPACES && opt.disabled);
  }

  /** The namespace to show: ?ns= if valid, else the stored choice, else the first owned, else the first usable. */
  function pickNamespace(options, { queryNs, storedNs } = {}) {
    const find = (name) => (name ? options.find((o) => o.namespace === name) : undefined);
    for (const cand of [find(queryNs), find(storedNs)]) if (usable(cand)) return cand;
    const owned = options.find((o) => o.role === "owner");
    if (owned) return owned;
    return options.find(usable);
  }

  function isOwner(ns) {
    return !!ns && ns.role === "owner";
  }

  // ---- menu ----------------------------------------------------------------------------------
  /** Browser href of a menu link: "/_" + path with {ns} substituted, ?ns=<current>, link fragment kept. */
  function menuHref(link, ns) {
    const frag = fragmentOf(link);
    let path = link.split("#")[0];
    if (ns && ns !== ALL_NAMESPACES) path = path.replace("{ns}", encodeURIComponent(ns));
    const q = ns ? queryString({ ns }) : "";
    return IFRAME_PREFIX + path + q + (frag !== undefined ? "#" + frag : "");
  }

  /** The menu link a browser location belongs to: longest link whose path+hash prefixes it. */
  function activeMenuLink(links, browserUrl, ns) {
    const u = parse(stripPrefix(browserUrl));
    const here = withSlash(u.path) + (u.hash ? u.hash.replace(/^#/, "") : "");
    let best = null, bestLen = -1;
    const flat = (links || []).flatMap((l) => (l.type === "section" ? l.items || [] : [l]));
    for (const l of flat) {
      let target = l.link;
      if (ns) target = target.replace("{ns}", ns);
      const lu = parse(target);
      const key = withSlash(lu.path) + (lu.hash ? lu.hash.replace(/^#/, "") : "");
      if (here.startsWith(key) && key.length > bestLen) {
        best = l;
        bestLen = key.length;
      }
    }
    return best;
  }

  // ---- iframe <-> browser URL mirroring --------------------------------------------------------
  /**
   * router: {url(): browser path+search+hash, navigate(path, params, fragment, replace)}
   * frame(): the iframe's Window (same origin) or null.
   */
  class IframeSync {
    constructor(router, frame, currentNs) {
      this.router = router;
      this.frame = frame;
      this.currentNs = currentNs || (() => "");
      this.src = "about:blank";
      this.lastSeen = undefined;
    }

    frameUrl() {
      const w = this.frame();
      if (!w || !w.location || !w.location.pathname) return undefined;
      return w.location.pathname + (w.location.search || "") + (w.location.hash || "");
    }

    /**
     * The browser navigated to `url` ("/_/app/..."). Returns the new iframe src, or null when the
     * iframe already shows that page (no reload). `forced` (menu click) always reloads: the origin
     * is prepended whenever the previous src lacked it so the value differs and the iframe reloads.
     */
    onNavigate(url, origin, forced) {
      const target = withSlash(stripPrefix(url));
      if (!forced && sameUrl(target, this.frameUrl())) return null;
      this.src = this.src.startsWith(origin) ? target : origin + target;
      return this.src;
    }

    /** Poll step: mirror a changed iframe location into the browser URL (under /_, ns kept). */
    tick() {
      const w = this.frame();
      const href = w && w.location ? w.location.href : undefined;
      if (href === undefined || href === this.lastSeen) return false;
      this.lastSeen = href;
      if (href === "about:blank") return false;
      const params = queryParams(w.location.search);
      if (!params.ns && this.currentNs()) params.ns = this.currentNs();
      const frag = w.location.hash ? w.location.hash.slice(1) : undefined;
      this.router.navigate(IFRAME_PREFIX + w.location.pathname, params, frag, false);  // history entry per app page
      return true;
    }
  }

  // ---- page state ----------------------------------------------------------------------------
  /** Which view a browser URL shows: home, iframe, manage-users, namespace-needed or not-found. */
  function viewFor(url) {
    const u = parse(url);
    const decoded = decodeURIComponent(u.path);
    if (u.path === "/" || u.path === "") return { page: "home" };
    if (u.path === "/manage-users" || u.path === "/manage-users/") return { page: "manage-users" };
    if (u.path === "/namespace-needed") return { page: "namespace-needed", path: queryParams(u.search).path || "" };
    if (u.path.startsWith(IFRAME_PREFIX + "/")) {
      if (decoded.includes("{ns}")) return { page: "namespace-needed", path: decoded };
      return { page: "iframe", src: stripPrefix(u.path) + u.search + u.hash };
    }
    return { page: "not-found", path: decoded };
  }

  // ---- renderers -----------------------------------------------------------------------------
  function renderSidenav(links, ns, browserUrl, build) {
    const active = viewFor(browserUrl).page === "home" ? null : activeMenuLink(links, browserUrl, ns);
    const home = `<a href="/${ns ? queryString({ ns }) : ""}" data-nav="1" class="${active ? "" : "active"}" data-cy-sidenav-menu-item="Home">Home</a>`;
    const items = (links || []).map((l) => {
      if (l.type === "section") {
        return `<div class="section"><span>${esc(l.text)}</span>${(l.items || []).map((i) =>
          `<a href="${esc(menuHref(i.link, ns))}" data-nav="1" class="${i === active ? "active" : ""}" data-cy-sidenav-menu-item="${esc(i.text)}">${esc(i.text)}</a>`).join("")}</div>`;
      }
      return `<a href="${esc(menuHref(l.link, ns))}" data-nav="1" class="${l === active ? "active" : ""}" data-cy-sidenav-menu-item="${esc(l.text)}">${esc(l.text)}</a>`;
    }).join("");
    const b = build || {};
    const footer = `<footer><span class="buildVersion">${esc((b.buildLabel || "Build") + " " + (b.buildVersion || "dev"))}</span>` +
      `<span class="buildId">${esc((b.buildLabel || "Build") + " " + (b.buildId || b.buildVersion || "dev"))}</span></footer>`;
    return home + items + footer;
  }

  function renderNamespaceSelector(options, current) {
    const real = options.filter((o) => o.namespace !== ALL_NAMESPACES);
    const label = real.length ? `${esc(current ? current.namespace : "")}${isOwner(current) ? ' <span class="owner">(Owner)</span>' : ""}` : NO_NAMESPACES;
    const opts = real.length
      ? options.map((o) => `<li data-cy-namespace="${esc(o.namespace)}" data-ns="${esc(o.namespace)}" class="${o.disabled ? "disabled" : ""}${current && o.namespace === current.namespace ? " selected" : ""}">` +
          `${esc(o.namespace)}${isOwner(o) ? ' <span class="owner">(Owner)</span>' : ""}</li>`).join("")
      : `<li class="disabled">${NO_NAMESPACES}</li>`;
    return `<button type="button" class="ns-trigger${real.length ? "" : " disabled"}" data-cy-selected-namespace>${label}</button><ul class="ns-menu" hidden>${opts}</ul>`;
  }

  function renderNotFound(path) {
    return `<div class="error-message-container"><div class="headline">404</div><div class="message">Sorry, <b>${esc(path)}</b> is not a valid page.</div>` +
      `<div class="back-to-home"><a href="/" data-nav="1" class="lib-link">back to home</a></div></div>`;
  }

  function renderNamespaceNeeded() {
    return `<div class="error-message-container"><div class="message">This page requires a namespace to be selected but no namespaces are currently available.</div>` +
      `<div class="back-to-home"><a href="/" data-nav="1" class="lib-link">back to home</a></div></div>`;
  }

  function dayLabel(d, now) {
    const day = (x) => new Date(x.getFullYear(), x.getMonth(), x.getDate()).getTime();
    const diff = Math.round((day(now) - day(d)) / 86400000);
    if (diff === 0) return "Today";
    if (diff === 1) return "Yesterday";
    return d.toLocaleDateString();
  }

  /** Events newest first, grouped under one heading per day (Today / Yesterday / date). */
  function renderActivities(events, now) {
    now = now || new Date();
    const ts = (e) => new Date(e.lastTimestamp || e.eventTime || (e.metadata || {}).creationTimestamp || 0);
    const sorted = [...(events || [])].sort((a, b) => ts(b) - ts(a));
    if (!sorted.length) return '<p class="message">No activities for this namespace.</p>';
    let html = "", cur = null;
    for (const e of sorted) {
      const d = ts(e), label = dayLabel(d, now);
      if (label !== cur) {
        html += `<h2>${esc(label)}</h2>`;
        cur = label;
      }
      const err = e.type && e.type !== "Normal";
      html += `<div class="activity-row"><span class="icon ${err ? "error" : "info"}">${err ? "error" : "info"}</span>` +
        `<span class="time">${esc(d.toLocaleTimeString())}</span><span class="obj">${esc((e.involvedObject || {}).name)}</span>` +
        `<span class="msg">${esc(e.message)}</span></div>`;
    }
    return html;
  }

  /** The five most recently active notebook servers (JWA list rows: {name, namespace, age, status}). */
  function recentNotebooks(rows, n) {
    const t = (r) => Date.parse(r.last_activity || r.age || "") || 0;
    return [...(rows || [])].sort((a, b) => t(b) - t(a) || String(a.name).localeCompare(String(b.name))).slice(0, n || 5);
  }

  const NS_RULE = /^[a-z0-9]([-a-z0-9]*[a-z0-9])?$/;
  const NS_RULE_MESSAGE = "Name can only start and end with alpha-num characters, dashes are only permitted between start and end. (minlength >= 1)";

  /** Default namespace for a new user: the e-mail's local part, DNS-label safe. */
  function suggestNamespace(user) {
    return String(user || "").split("@")[0].replace(/[^\w]|\./g, "-").replace(/^-+|-+$|_/g, "").toLowerCase();
  }

  function validateNamespace(name) {
    return NS_RULE.test(name || "") ? null : NS_RULE_MESSAGE;
  }

  /**
   * Registration: POST /api/workgroup/create, then poll /api/workgroup/exists until hasWorkgroup
   * (times x delayMs, 66 x 300 ms = 20 s by default). api: {create(ns), exists()} -> Promises.
   */
  async function register(api, name, { times = 66, delayMs = 300, sleep } = {}) {
    const bad = validateNamespace(name);
    if (bad) return { ok: false, error: bad };
    try {
      await api.create(name);
    } catch (e) {
      return { ok: false, error: e.message || String(e) };
    }
    const wait = sleep || ((ms) => new Promise((r) => setTimeout(r, ms)));
    for (let i = 0; i < times; i++) {
      try {
        const r = await api.exists();
        if (r && r.hasWorkgroup) return { ok: true };
      } catch (e) { /* profile not visible yet */ }
      await wait(delayMs);
    }
    return { ok: false, error: "Profile was created but is not available yet; try Finish again." };
  }

  /** Contributors table rows for the manage-users page (owner view; admins see every namespace). */
  function renderContributors(ns, users) {
    const rows = (users || []).map((u) => `<tr><td>${esc(u)}</td><td><button data-rm="${esc(u)}" data-ns="${esc(ns)}">remove</button></td></tr>`).join("");
    return rows ? `<table class="contributors">${rows}</table>` : '<p class="message">No contributors.</p>';
  }

  return {
    ALL_NAMESPACES, NO_NAMESPACES, ALL_NS_APPS, IFRAME_PREFIX, esc,
    withSlash, stripPrefix, queryParams, queryString, fragmentOf, sameUrl,
    allNamespacesAllowed, namespaceOptions, storageKey, pickNamespace, isOwner,
    menuHref, activeMenuLink, IframeSync, viewFor,
    renderSidenav, renderNamespaceSelector, renderNotFound, renderNamespaceNeeded, renderActivities,
    recentNotebooks, suggestNamespace, validateNamespace, register, renderContributors, NS_RULE_MESSAGE,
  };
});
